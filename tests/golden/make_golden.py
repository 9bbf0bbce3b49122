"""Generate tests/golden/*.npz from the CPU restatement (oracle/).

The reference holds no golden vectors and its CPU averager does not compile
as shipped ("Oracle"), so these fixtures pin the restatement
itself: they are regression vectors for the oracle and the GPU path, made
from the seeded counter-based generator (inputs are regenerated, only outputs
are stored).  Run:  python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

SEED = 0x5EED
FRAMES = 4096
GRADES = (1, 3, 7, 32, 41, 64, 1000, 1024)


def main():
    oracle.build()
    out = {}
    for C in (1, 2):
        x = oracle.synth_i16(FRAMES * C, seed=SEED)
        for k in GRADES:
            out[f"i16_C{C}_k{k}"] = oracle.mavg_i16(x, k, C)
        xf = oracle.synth_f32(FRAMES * C, seed=SEED, dist=1)
        for k in GRADES:
            out[f"f32u_C{C}_k{k}"] = oracle.mavg_f32(xf, k, C)
    np.savez_compressed(os.path.join(HERE, "mavg_golden.npz"), **out)
    # config #1 (BASELINE.json configs[0]): N=2^20, k=32 -- digests only
    x = oracle.synth_i16(1 << 20, seed=SEED)
    xf = oracle.synth_f32(1 << 20, seed=SEED)
    digests = {
        "i16_n1048576_C1_k32": hashlib.sha256(oracle.mavg_i16(x, 32, 1).tobytes()).hexdigest(),
        "f32_n1048576_C1_k32": hashlib.sha256(oracle.mavg_f32(xf, 32, 1).tobytes()).hexdigest(),
        "i16_n1048576_C2_k32": hashlib.sha256(oracle.mavg_i16(x, 32, 2).tobytes()).hexdigest(),
    }
    with open(os.path.join(HERE, "digests.txt"), "w") as f:
        for key in sorted(digests):
            f.write(f"{key} {digests[key]}\n")
    print("wrote", len(out), "vectors and", len(digests), "digests")


if __name__ == "__main__":
    main()
