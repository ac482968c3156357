# Kernel timeline + per-kernel PMC of one fusion workload (exp_fuse.py; default config 2:
# 256^3, 64 frames of 640x480) in the pipelined mode: where a call's time goes and what
# binds phase F / pass B there.  ARGS overrides the workload, TAG names the output.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${ARGS:---grid 256 --poses 64}
TAG=${TAG:-cfg2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/exp_fuse.py --tag $TAG $ARGS --calls 40 --modes pipelined > $OUT/kt.json 2> $OUT/kt.err || { echo KTFAIL; tail -5 $OUT/kt.err; exit 1; }
cat $OUT/kt.json
python3 tools/kt_timeline.py $OUT/kt 5 | head -20
i=0
for pmc in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- python3 tools/exp_fuse.py --tag $TAG $ARGS --calls 1 --modes serial > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { echo "PMCFAIL $pmc"; tail -5 $OUT/pmc$i.err; exit 2; }
  echo "pmc pass $i done"
done
python3 tools/pmc_dir.py $OUT | grep -E "k_bk_(fuse|pairs|rays)" || true
echo PROFOK
