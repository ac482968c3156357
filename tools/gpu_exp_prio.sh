# Stage order x issue priority x hardware queues A/B (experiment builds): pass A on its own
# stream (split), one staging stream per slot (slots), s_setprio(1) in B and F (prio) or F
# only (priof); name suffix _q8 = GPU_MAX_HW_QUEUES=8 (HIP's default 4 may map two of the
# volume's streams onto one hardware queue).  512^3 x 128 frames under a kernel trace
# (timeline), then config 2 (256^3 x 64) untraced.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_prio
mkdir -p $OUT
for name in ${PRIO_RUNS:-product product_q8 slots slots_q8 slots_priof slots_priof_q8 split_priof split prio split_prio}; do
  base=${name%_q8}
  q=4; [ "$base" != "$name" ] && q=8
  if [ "$base" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$base/libdmf.so; fi
  echo "== $name (hw queues $q)"
  GPU_MAX_HW_QUEUES=$q DMF_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o run -- python3 tools/exp_fuse.py --tag $name --calls 30 --modes pipelined > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; exit 1; }
  cat $OUT/$name.json
  python3 tools/kt_timeline.py $OUT/kt_$name 3 > $OUT/timeline_$name.txt 2>&1; tail -11 $OUT/timeline_$name.txt
  GPU_MAX_HW_QUEUES=$q DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_fuse.py --tag cfg2_$name --grid 256 --poses 64 --calls 60 --modes pipelined > $OUT/cfg2_$name.json 2> $OUT/cfg2_$name.err || { echo "FAIL cfg2 $name"; tail -5 $OUT/cfg2_$name.err; exit 2; }
  cat $OUT/cfg2_$name.json
done
echo PRIOOK
