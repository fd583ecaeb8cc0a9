# 8-rank rehearsals of the two 8-GPU flows on one GPU (every rank on cuda:0, gloo collectives):
#   config 4: torchrun 8 x bench.py --config 4 (N = 1e7 over 8 ranks) vs one process and the C oracle;
#   config 5 --single-chain: ONE chain at N = 8e6 over 8 ranks vs SeqNNGP's chain at N = 8e6, 25 iterations.
#   TAG=<tag> [PARTS="4 5"] bash tools/gpu_rehearse8.sh    -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${TAG:?set TAG}
mkdir -p $out
parts=${PARTS:-4 5}
if [[ " $parts " == *" 4 "* ]]; then
echo "[rehearse8] config 4, 8 ranks $(date +%T)"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 8 --config 4 --rehearse-on-one-gpu --steps 5 --warmup 2 --cpu-seconds 0 \
  > $out/config4_w8.json 2> $out/config4_w8.err || exit 1
echo "[rehearse8] config 4, one process + oracle $(date +%T)"
timeout -k 10 600 python tools/oracle_bench_config.py --config 4 > $out/config4_oracle.json 2> $out/config4_oracle.err || exit 1
fi
if [[ " $parts " == *" 5 "* ]]; then
echo "[rehearse8] config 5 single chain, 8 ranks $(date +%T)"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29582 bench.py --gpus 8 --config 5 --single-chain --rehearse-on-one-gpu --steps 25 \
  --warmup 0 --cpu-seconds 0 > $out/config5_single_w8.json 2> $out/config5_single_w8.err || exit 1
echo "[rehearse8] config 5 SeqNNGP at N = 8e6 $(date +%T)"
timeout -k 10 600 python bench.py --config 5 --n 8000000 --steps 25 --warmup 0 --cpu-seconds 0 \
  > $out/config5_seq_n8e6.json 2> $out/config5_seq_n8e6.err || exit 1
fi
echo "[rehearse8] done $(date +%T)"
