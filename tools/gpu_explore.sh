# quick exploration runs on the GPU box (bench variants + SQ counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/explore
B="timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0"
$B > gpurun_out/explore/lane_bf.json 2>>gpurun_out/explore/err.log || exit $?
$B --loglik-only > gpurun_out/explore/lane_ll.json 2>>gpurun_out/explore/err.log || exit $?
$B --m 10 > gpurun_out/explore/lane_m10.json 2>>gpurun_out/explore/err.log || exit $?
$B --m 8 > gpurun_out/explore/lane_m8.json 2>>gpurun_out/explore/err.log || exit $?
$B --kind matern32 --theta 1.0,17.320508075688772,0.1 --n 100000 --steps 50 > gpurun_out/explore/matern_1e5.json 2>>gpurun_out/explore/err.log || exit $?
$B --m 20 --n 1000000 --steps 5 > gpurun_out/explore/wave_m20.json 2>>gpurun_out/explore/err.log || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/explore/pmc_sq -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 > /dev/null 2>>gpurun_out/explore/err.log || exit $?
for f in gpurun_out/explore/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e9,3), 'Gloc/s', round(d['roofline']['kernel_ms'],4), 'ms', d['config']['m'], d['config']['write_BF'])"; done
