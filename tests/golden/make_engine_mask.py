"""Extract the reference's own engine-scene outputs as a data fixture.

Reads (in this container only; /root/reference does not travel to the GPU box)
    bindings/zombie/demo/scenes/engine/solutions/wost.pfm
    bindings/zombie/demo/scenes/engine/solutions/bvc.pfm
-- 256 x 256 "PF" images written by the reference's saveSolutionGrid /
saveEvaluationGrid (grid.h:272-350, 370-414) through Image<3>::writePFM
(image.h:173-198, rows bottom to top) -- and stores which grid points are non-zero,
indexed [i, j] for the grid point (i / 256, j / 256) of the scene's bounding box
(createSolutionGrid, grid.h:35-52; solution->get(j, i), grid.h:319,409).

Only the zero / non-zero pattern is kept (np.packbits), plus the raw values' sha256
for provenance.  Output: tests/golden/engine_solution_masks.npz.

    python tests/golden/make_engine_mask.py
"""
import hashlib
import os

import numpy as np

REF = "/root/reference/bindings/zombie/demo/scenes/engine/solutions"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "engine_solution_masks.npz")


def read_pf(path):
    raw = open(path, "rb").read()
    lines, pos = [], 0
    for _ in range(3):
        end = raw.index(b"\n", pos)
        lines.append(raw[pos:end].decode().strip())
        pos = end + 1
    assert lines[0] == "PF", lines
    w, h = map(int, lines[1].split())
    scale = float(lines[2])
    px = np.frombuffer(raw[pos:pos + 12 * w * h], "<f4" if scale < 0 else ">f4").reshape(h, w, 3)
    return px, hashlib.sha256(raw).hexdigest()


def main():
    out = {}
    for name in ("wost", "bvc"):
        px, sha = read_pf(os.path.join(REF, name + ".pfm"))
        g = px.shape[0]
        nonzero_rows = (px != 0).any(axis=2)          # file row r = image row g-1-r (writePFM flips)
        nonzero_ij = nonzero_rows[::-1].T             # [i, j]: image row j, column i
        out[name + "_nonzero_bits"] = np.packbits(nonzero_ij.ravel())
        out[name + "_sha256"] = np.array(sha)
        out["grid_res"] = np.array(g)
        print(f"{name}: {g}x{g}, non-zero {nonzero_ij.mean():.4%}, sha256 {sha[:16]}")
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
