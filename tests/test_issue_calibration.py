"""The calibrated VALU-issue figure (tools/collect_sq.py combine): every instruction type of the
mix passes weighted by its measured SIMD-cycles per wave64 instruction (tools/mb_latency issue),
the untyped remainder at the move / select cost; bench.py reports it when the committed
profile carries it (and the uncalibrated 4-cycle figure only as frac_4cyc)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _mb(cyc):
    return {"results": [{"op": op, "waves_per_simd": w, "simd_cycles_per_wave_instr": c * (4 / w if w < 4 else 1)}
                        for op, c in cyc.items() for w in (1, 2, 4)]}


def test_weighted_issue_sums_types_at_their_cost():
    import collect_sq as cs
    cyc = {op: 2.0 for op in set(cs.TYPE_OPS.values()) | set(cs.OTHER_OPS)}
    cyc["v_cndmask_b32"] = 5.0
    cyc.update({"v_fma_f64": 4.0, "v_mul_f64": 4.0, "v_add_f64": 4.0, "v_rcp_f64": 8.0, "v_exp_f32": 4.0})
    got = cs.issue_cycles(_mb(cyc))
    assert got == cyc  # the 4-waves-per-SIMD column
    t = 1e-3
    simd_cycles = t * cs.CLOCK_HZ * cs.SIMDS
    issue = {"counters": {"SQ_INSTS_VALU": 1000.0}, "kernel_s": t}
    mix = {"counters": {"SQ_INSTS_VALU_FMA_F64": 100.0, "SQ_INSTS_VALU_TRANS_F64": 10.0, "SQ_INSTS_VALU_INT32": 200.0}}
    mix2 = {"counters": {"SQ_INSTS_VALU_FMA_F32": 300.0}}
    frac, parts, other = cs.weighted_issue(issue, mix, mix2, cyc)
    assert other == 1000.0 - 610.0
    busy = 100 * 4.0 + 10 * 8.0 + 200 * 2.0 + 300 * 2.0 + 390 * 2.0
    assert frac == pytest.approx(busy / simd_cycles)
    assert sum(parts.values()) == pytest.approx(frac)
    # the CDNA3 rule of thumb would have charged every instruction 4 cycles
    assert frac < 1000 * 4 / simd_cycles
    hi, _, _ = cs.weighted_issue(issue, mix, mix2, cyc, other_op="v_cndmask_b32")
    assert hi == pytest.approx((busy + 390 * 3.0) / simd_cycles)
