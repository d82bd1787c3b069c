for v in pw; do
STAMPS_LIB=tools/libVS_$v.so timeout -k 10 200 python3 tools/stamps.py random 4096 > gpurun_out/ex_$v.log 2>&1 || exit 1
STAMPS_LIB=tools/libVS_$v.so timeout -k 10 200 python3 tools/stamps.py mix 4096 > gpurun_out/ex_${v}_mix.log 2>&1 || exit 1
done
