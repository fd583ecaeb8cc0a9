# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box via gpurun).
#   bash tools/profile.sh <tag> [bench args...]
# kernel trace + stats in one run; PMC counters in separate passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950; no --pmc together with trace domains).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r01}; shift
out=gpurun_out/prof_$tag
mkdir -p $out
args="--steps 20 --warmup 3 --cpu-seconds 0 $*"
echo "$args" > $out/args.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/trace_bench.json 2> $out/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- python3 bench.py $args > $out/pmc_fetch_bench.json 2> $out/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- python3 bench.py $args > $out/pmc_write_bench.json 2> $out/pmc_write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d $out/pmc_sq -o run -- python3 bench.py $args > $out/pmc_sq_bench.json 2> $out/pmc_sq.err || exit $?
python3 tools/summarize_profile.py $tag && cp -r profiles/$tag $out/summary
