# N-rank rehearsal of the bench on one GPU (every rank on cuda:0, gloo collectives; via gpurun):
# 2 and 4 ranks at 1e6 locations per rank, and the one-process run at the same total N for the
# log-likelihood comparison -> gpurun_out/${TAG}
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${TAG:-rehearse}
mkdir -p $out
for w in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29500 + w)) bench.py --gpus $w --rehearse-on-one-gpu --steps 20 --warmup 5 --cpu-seconds 0 \
    > $out/bench_w$w.json 2> $out/bench_w$w.err || exit 1
  timeout -k 10 300 python bench.py --n $((w * 1000000)) --steps 20 --warmup 5 --cpu-seconds 0 \
    > $out/bench_one_n${w}e6.json 2> $out/bench_one_n${w}e6.err || exit 1
done
