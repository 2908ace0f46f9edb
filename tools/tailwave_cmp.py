"""Compare two tools/tailwave_diag.py dumps level by level: for every
variable, the number of stored cells that differ and the largest difference
(cells the device does not store, edge and corner ghosts, are skipped).

    python tools/tailwave_cmp.py a.npz b.npz
"""
import sys

import numpy as np


def stored(nc):
    s = nc + 2
    ix = np.arange(s)
    bnd = ((ix == 0) | (ix == s - 1)).astype(int)
    return (bnd[:, None, None] + bnd[None, :, None] + bnd[None, None, :]) < 2


def main():
    a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
    print("max_res", float(a["max_res"][0]), float(b["max_res"][0]))
    keys = sorted((k for k in a.files if "@" in k), key=lambda k: (int(k.split("@")[1]), k))
    for k in keys:
        x, y = a[k], b[k]
        m = stored(x.shape[-1] - 2)
        d = np.abs(x[:, m] - y[:, m])
        nd = int(np.count_nonzero(x[:, m].view(np.uint64) != y[:, m].view(np.uint64)))
        print(f"{k:10s} boxes {x.shape[0]:5d}  differing cells {nd:8d}  max |diff| {float(d.max()):.3e}")


if __name__ == "__main__":
    main()
