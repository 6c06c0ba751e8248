"""BASELINE config 1: one UDP flow PERIODIC [1000 1024] over loopback for
10 s (doc/example.mgn:9 + LISTEN), through the batched socket layer (include/mgenx_io.hpp:
sendmmsg / recvmmsg).  Plumbing: every one of the 10,000 messages arrives once, in sequence
order 0..9999, intact (CRC checked), with the fields and tx times it was sent with.
CPU: packed and decoded by the oracle restatement (the reference's CPU path, no GPU).
GPU: packed and decoded by libmgenx (GPU pack, GPU unpack + CRC) around the same sockets."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "loopback")


def _run(mode, count, rate, size, *extra):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", ROOT, "tests/cpp/loopback"], check=True)
    r = subprocess.run([BIN, mode, str(count), str(rate), str(size), *extra],
                       capture_output=True, text=True, timeout=120)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["ok"], r.stdout + r.stderr
    return out


def test_config1_periodic_1000_1024_cpu_path():
    out = _run("cpu", 10000, 1000, 1024)
    assert out["received"] == 10000 and out["lost"] == 0
    assert 9.5 < out["elapsed_s"] < 15.0          # PERIODIC 1000/s for 10 s


@pytest.mark.gpu
def test_config1_periodic_1000_1024_gpu_path():
    out = _run("gpu", 10000, 1000, 1024)
    assert out["received"] == 10000 and out["lost"] == 0


def test_ipv6_loopback_cpu_path():
    """The socket layer over IPv6 (::1): sources reported as IPv6, dst carried as IPv6."""
    out = _run("cpu", 3000, 3000, 700, "v6")
    assert out["received"] == 3000 and out["lost"] == 0 and out["v6"]


@pytest.mark.gpu
@pytest.mark.parametrize("v6", [False, True])
def test_recv_ring_gpu_path(v6):
    """RecvRing: 20,000 datagrams at 20,000/s decoded on the GPU batch by batch during the run
    (pinned stages on their own streams), every one checked in order."""
    out = _run("ring", 20000, 20000, 512, *(["v6"] if v6 else []))
    assert out["received"] == 20000 and out["lost"] == 0 and out["ring_stages"] > 10
