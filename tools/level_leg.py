"""Diagnostic: bench.py's level leg alone (C3 mix chunks at one level: GB/s, ratio, K1 / entropy
ms per launch, libzstd decode of every frame).  usage: python3 tools/level_leg.py LEVEL [CHUNKS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

level = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.CHUNKS
host = bench.gen_chunks("mix", n, 0)
r = bench.level_leg(host, torch.device("cuda", 0), level, 8, None)
print(json.dumps({"level": level, "chunks": n, **{k: r[k] for k in ("value", "ms_per_step", "ratio", "libzstd_verified")},
                  "kernel_ms": r["roofline"]["kernel_ms"]}))
