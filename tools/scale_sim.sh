for c in 2048 4096 8192; do timeout -k 10 120 python bench.py --chunks $c --no-legs --no-decompress --no-cpu-baseline --no-verify > gpurun_out/sc_$c.json 2>/dev/null || exit 1; done
