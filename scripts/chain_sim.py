"""CPU model of the scan's chain hypothesis (mgenx_scan.hip, scan_chain_*): on a TCP stream
built by the oracle's transmit restatement (config 5's shape, fewer records), compute the
candidates by the detect rule, the level-1 / level-2 marks and the chain check, and compare the
accepted set with the oracle's sequential framing.  Usage: python scripts/chain_sim.py [n] [rf]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from mgen_amd._abi import DESC_DTYPE  # noqa: E402
from mgen_amd.workloads import make_templates  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
rf = len(sys.argv) > 2 and sys.argv[2] == "1"
tmpl, pool = make_templates(64)
desc = np.zeros(n, DESC_DTYPE)
seq = np.arange(n)
desc["tmpl"] = seq % 64
desc["seq_num"] = seq
desc["tx_sec"] = 1_700_000_000
desc["tx_usec"] = seq % 1_000_000
desc["flags"] = 4
s = O.tcp_tx_batch(tmpl, desc, np.full(n, 16384, np.uint32), pool, checksum=True, random_fill=rf)
N = len(s)
p = np.arange(N - 3, dtype=np.int64)
L = (s[:-3].astype(np.int64) << 8) | s[1:-2]
cand = p[(s[2:-1] == 2) & (L >= 4) & (p + L <= N)]
Lc = (s[cand].astype(np.int64) << 8) | s[cand + 1]
succ = cand + Lc
cset = set(cand.tolist())


def is_copy(q):
    return q >= 8192 and q + 16 <= N and bytes(s[q:q + 16]) == bytes(s[q - 8192:q - 8192 + 16])


copy = np.array([is_copy(int(q)) for q in cand])
m1 = set(succ[(~copy) & (succ + 2 <= N)].tolist())
h1 = np.array([q == 0 or q in m1 for q in cand.tolist()])
m2 = set(succ[h1 & (succ + 2 <= N)].tolist())
H = [q for q in cand.tolist() if q == 0 or q in m2]
ok = len(H) > 0 and H[0] == 0
for i in range(len(H) - 1):
    hq = H[i]
    if hq + ((int(s[hq]) << 8) | int(s[hq + 1])) != H[i + 1]:
        ok = False
        print("break at", i, hq, H[i + 1])
        break
last = H[-1]
nxt = last + ((int(s[last]) << 8) | int(s[last + 1]))
ok = ok and nxt not in cset
ref = O.tcp_scan(bytes(s))
print("bytes", N, "candidates", len(cand), "copies", int(copy.sum()), "H", len(H), "ok", ok,
      "oracle records", len(ref[0]) if isinstance(ref, tuple) else ref)

# the one-scatter form: each level-1 mark keeps its marker's length (q - p); a position marked
# by two different candidates keeps none (then taken into H on doubt: the check proves H)
pred = {}
for p0, q0, c0 in zip(cand.tolist(), succ.tolist(), copy.tolist()):
    if c0 or q0 + 2 > N:
        continue
    pred[q0] = q0 - p0 if q0 not in pred or pred[q0] == q0 - p0 else 0
multi = sum(1 for v in pred.values() if v == 0)
H2 = [q for q in cand.tolist() if q == 0 or (q in pred and (pred[q] == 0 or q - pred[q] == 0
                                                             or (q - pred[q]) in pred))]
print("one-scatter H", len(H2), "same as level-2 H", H2 == H, "multi-marked", multi)
