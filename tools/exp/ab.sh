# A/B bench runs: tools/exp/ab.sh TAG STEPS "LIB|KNOBS" ...  LIB: lib/exp/libLIB.so ("" = the
# release library), KNOBS: FFV1HIP_DEBUG ("" = none); variants run interleaved twice
cd $GRAFT_REPO_ROOT
T=$1; S=$2; shift 2
mkdir -p gpurun_out/$T
i=0
for rep in 1 2; do
for v in "$@"; do
  i=$((i+1))
  lib=${v%%|*}; kn=${v#*|}
  L=""; [ -n "$lib" ] && L=$GRAFT_REPO_ROOT/ffmpeg-ffv1-p-frames_amd/lib/exp/lib$lib.so
  FFV1HIP_LIB=$L FFV1HIP_DEBUG=$kn timeout -k 10 300 python bench.py --steps $S --warmup 3 --no-cpu-baseline --no-decode-check > gpurun_out/$T/b$i.json 2>gpurun_out/$T/b$i.err || { tail -5 gpurun_out/$T/b$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/$T/b$i.json').read().strip().splitlines()[-1]);k=d['kernel_ms_per_step'];print('[$v]',d['value'],d['ms_per_step'],'oracle',d['bitexact_vs_oracle']['equal'],'pin',d['bitexact_vs_reference_pin'],' '.join('%s=%.1f'%(a.replace('ffv1_',''),b) for a,b in k.items() if a!='launches'))"
done
done
