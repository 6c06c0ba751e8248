#!/bin/bash
# round 6: analytics parity, config-4 A/B, kernel trace, phase cycles
set -u
export TMPDIR=/tmp
bash scripts/r06_an.sh || exit 1
timeout -k 10 300 python3 scripts/skel_prof.py || exit 1
