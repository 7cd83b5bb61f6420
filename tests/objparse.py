"""Independent OBJ reader for the tests (restates the reference's parsing rules):
2D  bindings/zombie/demo/scene.h:104-145  (`v x y`, `l i j`, flipOrientation swaps ends)
3D  fcpw/utilities/scene_loader.inl:100-150 (`v x y z`, `f a[/b/c] ...` flattened in triples)
Used to pin the product's C++ parser and to feed the oracle."""
import numpy as np


def load(path, dim, flip=False):
    vs, ix = [], []
    with open(path) as f:
        for line in f:
            t = line.split()
            if not t:
                continue
            if t[0] == "v":
                vs.append([np.float32(c) for c in t[1:1 + dim]])
            elif dim == 2 and t[0] == "l":
                i, j = int(t[1]) - 1, int(t[2]) - 1
                ix.append([j, i] if flip else [i, j])
            elif dim == 3 and t[0] == "f":
                for tok in t[1:]:
                    ix.append(int(tok.split("/")[0]) - 1)
    v = np.asarray(vs, np.float32).reshape(-1, dim)
    if dim == 3:
        ix = np.asarray(ix, np.int32).reshape(-1, 3)
    else:
        ix = np.asarray(ix, np.int32).reshape(-1, 2)
    return v, ix
