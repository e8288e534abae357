#!/bin/bash
# Several A/B groups in one GPU call: tools/exp/ab_multi.sh TAG STEPS "BENCH ARGS|LIB LIB ..." ...
# LIB "-" = the release library; each group's variants run interleaved twice
cd $GRAFT_REPO_ROOT
T=$1; S=$2; shift 2
mkdir -p gpurun_out/$T
i=0
for grp in "$@"; do
  A=${grp%%|*}; libs=${grp#*|}
  for rep in 1 2; do
    for lib in $libs; do
      i=$((i+1))
      L=""; [ "$lib" != "-" ] && L=$GRAFT_REPO_ROOT/ffmpeg-ffv1-p-frames_amd/lib/exp/lib$lib.so
      FFV1HIP_LIB=$L timeout -k 10 300 python bench.py $A --steps $S --warmup 3 --no-cpu-baseline --no-decode-check > gpurun_out/$T/b$i.json 2>gpurun_out/$T/b$i.err || { tail -5 gpurun_out/$T/b$i.err; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/$T/b$i.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('[$A][$lib]',d['value'],d['ms_per_step'],'oracle',d['bitexact_vs_oracle']['equal'],' '.join('%s=%.1f'%(a.replace('ffv1_',''),b) for a,b in k.items() if a!='launches'))"
    done
  done
done
