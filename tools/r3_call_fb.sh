#!/bin/bash
# 2D first balls: the uniform-ball cooperative sampler (xcoop) against the per-lane loop (xb),
# bit-exact dumps + timings; then timing-only attribution variants of the first-ball sections
# (xnoperm: no stratified-sample shuffle, xnosmp: no rejection loop, xnobes: no fused Bessels)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
bash tools/ab_generic.sh fb1 "xb xcoop" &&
ROUNDS=2 timeout -k 10 500 bash tools/ab.sh "xb xnoperm xnosmp xnobes" "B_karman64k C_dirichlet512" > gpurun_out/fb1_attr.log 2>&1
