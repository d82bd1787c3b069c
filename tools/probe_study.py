"""Ratio of oracle frames (= GPU frames) vs libzstd L3 on 64 KiB chunks that start with a
random prefix (the incompressibility probe's ratio cliff).  CPU only."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import zh_testlib as T

def main(n=16):
    rng = np.random.default_rng(5)
    for kind in ("text", "json", "mix", "csv", "source"):
        for pre in (0, 1024, 2048, 3000, 4096, 6144, 8192, 16384, 32768):
            o = z = 0
            worst = 9.0
            for i in range(n):
                c = T.gen(T.KINDS[kind], 1, 100 + i, 65536).copy()
                c[:pre] = rng.integers(0, 256, pre, dtype=np.uint8)
                a = len(T.oracle_frame(c)); b = len(T.zstd_compress(c, 3))
                o += a; z += b
                worst = min(worst, b / a)
            print(f"{kind:6s} prefix {pre:5d}: oracle {n*65536/o:6.3f} libzstd {n*65536/z:6.3f} ratio-of-ratios {z/o:5.3f} worst chunk {worst:5.3f}")
    # random
    c = rng.integers(0, 256, 65536 * 8, dtype=np.uint8)
    print("random frames", [len(T.oracle_frame(c[i*65536:(i+1)*65536])) for i in range(8)])

if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 16)
