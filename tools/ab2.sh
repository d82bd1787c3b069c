#!/bin/bash
# A/B over datasets on one GPU box: A = tools/libA.so, B = tools/libB.so (tools/ab_build.sh REV),
# variants tools/libV_<X>.so named in $VARIANTS.  K1 parity tests on B first ($TESTS).  Output under
# gpurun_out/TAG_*.   usage (box): bash tools/ab2.sh TAG "random mix"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$R/custom-nvcomp-with-zstd_amd
TAG=${1:-ab2}
DS=${2:-"random mix"}
mkdir -p $R/gpurun_out
if [ -n "$TESTS" ]; then
  CUDA_ZSTD_HIP_LIB=$R/tools/libB.so timeout -k 10 400 python3 -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/${TAG}_testsB.log 2>&1 || { tail -30 $R/gpurun_out/${TAG}_testsB.log; exit 1; }
  echo "tests B: $(tail -1 $R/gpurun_out/${TAG}_testsB.log)"
fi
for ds in $DS; do
  for k in $(seq 1 ${ROUNDS:-2}); do
    for v in A B $VARIANTS; do
      if [ $v = A ]; then L=$R/tools/libA.so; elif [ $v = B ]; then L=$R/tools/libB.so; else L=$R/tools/libV_$v.so; fi
      CUDA_ZSTD_HIP_LIB=$L timeout -k 10 200 python3 $R/bench.py --dataset $ds --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/${TAG}_${ds}_${v}${k}.json 2>/dev/null
      python3 -c "import json; d=json.loads(open('$R/gpurun_out/${TAG}_${ds}_${v}${k}.json').read().strip().splitlines()[-1]); print('$ds $v', d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['ratio'])"
    done
  done
done
# SQ instruction mix of every library on each dataset ($SQ = datasets): one rocprofv3 --pmc pass each
for ds in $SQ; do
  for v in A B $VARIANTS; do
    if [ $v = A ]; then L=$R/tools/libA.so; elif [ $v = B ]; then L=$R/tools/libB.so; else L=$R/tools/libV_$v.so; fi
    export CUDA_ZSTD_HIP_LIB=$L
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      --kernel-trace -d $R/gpurun_out/prof_sq_${TAG}_${ds}_$v/a -o run --output-format csv -- python3 $R/bench.py --dataset $ds --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-decompress --no-legs > $R/gpurun_out/${TAG}_sq_${ds}_$v.log 2>&1) || { echo "sq $ds $v failed"; exit 2; }
    unset CUDA_ZSTD_HIP_LIB
    python3 $R/tools/sq_summary.py ${TAG}_${ds}_$v > /dev/null && python3 -c "import json; d=json.load(open('$R/profiles/${TAG}_${ds}_${v}_sq_summary.json'))['kernels'].get('zh_lz_kernel', {}); print('sq $ds $v', d.get('valu_insts_per_input_byte'), d.get('valu_issue_frac'), d.get('salu_per_valu'), d.get('lds_bank_conflict_frac'), round(d.get('kernel_cycles', 0)))"
  done
done
for ds in $STAMPS; do
  STAMPS_LIB=$R/tools/libBS.so timeout -k 10 200 python3 $R/tools/stamps.py $ds 4096 > $R/gpurun_out/${TAG}_stampsB_$ds.log 2>&1 || true
done
echo ab2-done
