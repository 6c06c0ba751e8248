"""CPU: the oracle reproduces the committed golden vectors (tests/golden/udp_matrix.npz)
and the C-ABI library loads and exports every symbol include/mgenx.h declares."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "udp_matrix.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD, allow_pickle=False))


def test_oracle_reproduces_pack_vectors(oracle, gold):
    sb = int(gold["slab_bytes"][0])
    for ck in (0, 1):
        for rf in (0, 1):
            slab, lens = oracle.udp_pack_batch(gold["tmpl"], gold["desc"], gold["pool"], sb,
                                               rec_off=gold["offs"], checksum=bool(ck),
                                               random_fill=bool(rf),
                                               fill_time=int(gold["fill_time"][0]))
            assert np.array_equal(slab, gold[f"pack_slab_ck{ck}_rf{rf}"])
            assert np.array_equal(lens, gold[f"pack_lens_ck{ck}_rf{rf}"])


def test_oracle_reproduces_unpack_vectors(oracle, gold):
    n = len(gold["unpack_lens"])
    for mode, force, tcp in (("udp", 0, 0), ("udp_force", 1, 0), ("tcp_force", 1, 1)):
        f = oracle.udp_recv_batch(gold["unpack_slab"], n, rec_off=gold["unpack_offs"],
                                  rec_len=gold["unpack_lens"], force=bool(force), tcp=bool(tcp))
        assert np.array_equal(f, gold[f"unpack_fields_{mode}"]), mode


def test_golden_covers_every_error_class(gold):
    errs = set(np.unique(gold["unpack_fields_udp_force"]["err"]).tolist())
    assert {0, 1, 2, 3, 4} <= errs
    # Pack returns 0 exactly for an unsupported dst type (mgenMsg.cpp:146-148) or a msg_len
    # short of the dst section (:207-210)
    tmpl, desc = gold["tmpl"], gold["desc"]
    t = tmpl[desc["tmpl"]]
    host_len = np.where(np.isin(t["host_type"], (1, 2)), t["host_len"], 0)
    failed = (~np.isin(t["dst_type"], (1, 2))) | (
        (desc["msg_len"] < 24 + t["dst_len"].astype(int) + host_len + 4) &
        (desc["msg_len"] < 24 + t["dst_len"].astype(int)))
    for key in ("pack_lens_ck0_rf0", "pack_lens_ck1_rf0", "pack_lens_ck1_rf1"):
        lens = gold[key]
        assert np.array_equal(lens == 0, failed), key
        assert np.array_equal(lens[~failed], desc["msg_len"][~failed]), key
    # truncation boundaries are present: records with hdr_len < 48 exist
    f = gold["unpack_fields_udp"]
    assert ((f["hdr_len"] > 0) & (f["hdr_len"] < 48)).any()
    assert (gold["unpack_fields_tcp_force"]["flags"] & 0x10).any()


def _header_functions():
    text = open(os.path.join(ROOT, "include", "mgenx.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mgenx_[a-z0-9_]+)\s*\(", text)))


def test_capi_library_exports_header_symbols():
    from mgen_amd import LIB_PATH, load
    assert os.path.exists(LIB_PATH), "libmgenx.so not built (run __graft_entry__.build())"
    lib = load()
    missing = [s for s in _header_functions() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.mgenx_abi_version() == 1


def test_python_symbol_list_matches_header():
    from mgen_amd import EXPORTED_SYMBOLS
    assert sorted(EXPORTED_SYMBOLS) == _header_functions()


def test_diagnostics_are_not_in_the_product_library():
    """mgenx_diag.h symbols live only in libmgenx_diag.so (the product ABI is mgenx.h)."""
    from mgen_amd import DIAG_LIB_PATH, DIAG_SYMBOLS, load
    text = open(os.path.join(ROOT, "include", "mgenx_diag.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    declared = sorted(set(re.findall(r"\b(mgenx_[a-z0-9_]+)\s*\(", text)))
    assert declared == sorted(DIAG_SYMBOLS)
    prod = ctypes.CDLL(os.path.join(ROOT, "mgen_amd", "libmgenx.so"))
    assert not [s for s in DIAG_SYMBOLS if hasattr(prod, s)]
    assert os.path.exists(DIAG_LIB_PATH)
    diag = load(diag=True)
    assert all(hasattr(diag, s) for s in DIAG_SYMBOLS + tuple(_header_functions()))


def test_capi_rejects_bad_arguments_without_gpu():
    from mgen_amd import load
    lib = load()
    # null ctx / null out are argument errors, detected before any HIP call
    assert lib.mgenx_ctx_create(0, None) == -1
    assert lib.mgenx_unpack_batch(None, None, 0, None, 0, None, 0, 1, None, 0, None) == -1
    assert lib.mgenx_pack_batch(None, None, None, None, 1, None, None, 0, None, 0, None, 0, 0,
                                None) == -1


def test_abi_struct_layouts_match_header(tmp_path):
    """Compile a probe against include/mgenx.h and compare offsets with the numpy mirrors."""
    from mgen_amd._abi import DESC_DTYPE, TMPL_DTYPE, MgenxCols
    src = tmp_path / "probe.c"
    fields_t = [n for n in TMPL_DTYPE.names]
    fields_d = [n for n in DESC_DTYPE.names]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mgenx.h"', 'int main(){']
    lines.append('printf("%zu %zu %zu\\n", sizeof(mgenx_flow_tmpl), sizeof(mgenx_pack_desc),'
                 ' sizeof(mgenx_cols));')
    for f in fields_t:
        lines.append(f'printf("t {f} %zu\\n", offsetof(mgenx_flow_tmpl, {f}));')
    for f in fields_d:
        lines.append(f'printf("d {f} %zu\\n", offsetof(mgenx_pack_desc, {f}));')
    for f, _ in MgenxCols._fields_:
        lines.append(f'printf("c {f} %zu\\n", offsetof(mgenx_cols, {f}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    import subprocess
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    st, sd, sc = map(int, out[0].split())
    assert st == TMPL_DTYPE.itemsize and sd == DESC_DTYPE.itemsize
    assert sc == ctypes.sizeof(MgenxCols)
    for line in out[1:]:
        if not line:
            continue
        kind, name, off = line.split()
        if kind == "t":
            assert TMPL_DTYPE.fields[name][1] == int(off), name
        elif kind == "d":
            assert DESC_DTYPE.fields[name][1] == int(off), name
        else:
            assert getattr(MgenxCols, name).offset == int(off), name
