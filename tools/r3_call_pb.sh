#!/bin/bash
# 2D first balls with the ball's Bessel members from the point-setup kernel (pb) against the
# shipped sources (b5): bit-exact dumps on B, C, D, then latency probe and config timings
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
ROUNDS=3 bash tools/ab_generic.sh pb1 "b5 pb"
