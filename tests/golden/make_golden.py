"""Generates tests/golden/products.json (committed).  Inputs are regenerable
from (n, seed) with the splitmix64/xoshiro256** stream shared by the product
(mpfft_fill_random) and the oracle (orc_fill_random).

Expected outputs are the exact products: Python int multiplication for the
small and C0/C1 shapes (independent of GMP), GMP mpn_mul -- the reference's own
integration-test oracle (mul_fft.c:5542) -- for the 10^9-bit configs.
Run: python tests/golden/make_golden.py [--big]        (everything; --big adds C2-C4)
     python tests/golden/make_golden.py --add C4       (compute only the named entries and
                                                       merge them into products.json)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import oracle as O  # noqa: E402

SMALL = [  # name, depth, w, n1, n2, seed1, seed2
    ("d6w1", 6, 1, 28, 28, 0x11, 0x12),
    ("d7w2_unbal", 7, 2, 120, 3, 0x21, 0x22),
    ("d8w1", 8, 1, 118, 118, 0x31, 0x32),
    ("d9w5", 9, 5, 1270, 1, 0x41, 0x42),
    ("d10w3", 10, 3, 1490, 1490, 0x51, 0x52),
    ("d11w1", 11, 1, 2030, 2030, 0x61, 0x62),
    ("d4w4", 4, 4, 1, 1, 0x71, 0x72),
]
BIG = [
    ("C0", 11, 1, 16384, 16384, 0x1001, 0x2002),
    ("C1", 11, 8, 261952, 261952, 0x1001, 0x2002),
]
HUGE = [
    ("C2", 15, 4, 15625000, 15625000, 0x1001, 0x2002),
    ("C3", 15, 4, 20312500, 20312500, 0x1001, 0x2002),
    # BASELINE configs[4]: the 10^10-bit north-star multiply (GMP mpn_mul: ~3 min, 5 GB of RAM)
    ("C4", 17, 2, 156250000, 156250000, 0x1001, 0x2002),
]


def as_int(a):
    return int.from_bytes(np.ascontiguousarray(a).tobytes(), "little")


def main():
    out = []
    todo = SMALL + BIG + (HUGE if "--big" in sys.argv else [])
    path = os.path.join(HERE, "products.json")
    if "--add" in sys.argv:
        names = set(sys.argv[sys.argv.index("--add") + 1].split(","))
        todo = [c for c in SMALL + BIG + HUGE if c[0] in names]
        with open(path) as f:
            out = [c for c in json.load(f) if c["name"] not in names]
    for name, depth, w, n1, n2, s1, s2 in todo:
        a = O.fill_random(n1, s1)
        b = O.fill_random(n2, s2)
        if name in ("C2", "C3", "C4"):
            r = O.gmp_mul(a, b)
            src = "gmp mpn_mul"
        else:
            v = as_int(a) * as_int(b)
            r = np.frombuffer(v.to_bytes(8 * (n1 + n2), "little"), dtype=np.uint64)
            src = "python int"
        c = {"name": name, "depth": depth, "w": w, "n1": n1, "n2": n2, "seed1": hex(s1), "seed2": hex(s2),
             "sha256": hashlib.sha256(r.tobytes()).hexdigest(), "source": src}
        if n1 + n2 <= 4200:
            c["product_hex"] = format(as_int(r), "x")
        out.append(c)
        print(name, c["sha256"][:16], src, flush=True)
    order = [c[0] for c in SMALL + BIG + HUGE]
    out.sort(key=lambda c: order.index(c["name"]))
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
