"""Builders for MGEN_DATA payload items in the reference's own encodings (test
infrastructure): MgenFlowCommand::SetStatus (mgenPayload.cpp:276-318), reports via the
oracle's restatement of MgenAnalytic's report_msg, and generic items."""
import numpy as np


def flow_command(statuses):
    """The item SetStatus builds for {flow_id: status} (len = 4 + 4N, N from the largest
    flow id; 'lo' mask then 'hi' mask, MSB first)."""
    maxf = max(statuses) if statuses else 0
    N = (2 * maxf - 16 - 1) // 32 + 1 if 2 * maxf > 16 else 0
    length = 2 + 2 + N * 4
    b = bytearray(length)
    b[0], b[1] = 1, length
    half = (length - 2) // 2
    for f, st in statuses.items():
        i = f - 1
        if st & 1:
            b[2 + (i >> 3)] |= 0x80 >> (i & 7)
        if st & 2:
            b[2 + half + (i >> 3)] |= 0x80 >> (i & 7)
    return bytes(b)


def addr(rng, v6=None):
    from oracle import oracle as O
    a = np.zeros(1, O.ADDR_DTYPE)
    v6 = rng.random() < 0.3 if v6 is None else v6
    a["type"], a["len"] = (2, 16) if v6 else (1, 4)
    a["port"] = rng.integers(0, 65536)
    a["addr"][0, :16 if v6 else 4] = rng.integers(0, 256, 16 if v6 else 4)
    return a


def random_values(rng):
    """Report doubles across the quantizers' ranges and edges."""
    dur = float(rng.choice([0.0, 1e-7, 5e-7, 1e-6, 1.7e-6, 0.001, 0.5, 1.0, 1.97, 9.99, 60.0,
                            599.9, 660.0, 700.0, rng.uniform(0, 700)]))
    ave = float(rng.choice([-1.0, -0.002, 0.0, 1e-7, 0.000119, 0.01, 2.5, rng.uniform(-1, 5)]))
    mn = ave - float(rng.choice([0.0, 1e-6, 0.0003, rng.uniform(0, 1)]))
    mx = ave + float(rng.choice([0.0, 1e-6, 0.0004, rng.uniform(0, 1)]))
    rate = float(rng.choice([0.0, -3.0, 0.05, 0.5, 1.0, 9.999, 10.0, 99.99, 1250.0, 1e6,
                             123456789.0, 10.0 ** rng.uniform(-3, 12)]))
    loss = float(rng.choice([0.0, 1e-6, 0.5 / 65535, 0.01, 0.5, 1.0, 1.2, rng.uniform(0, 1)]))
    return dur, ave, mn, mx, rate, loss
