# Roofline provenance for every bench preset (run on the GPU box via gpurun):
#   TAG=<tag> bash tools/gpu_provenance.sh [presets...]      (default presets: 3 2 4 5)
# Per preset: one rocprofv3 --kernel-trace --stats run, then separate --pmc passes (FETCH_SIZE,
# WRITE_SIZE, the VALU class counters, the VALU-busy counters) -- no pass mixes --pmc with a trace
# domain, each stays inside the per-block counter limits (8 SQ, <= 4 TCC, 1 GRBM).  Output:
# gpurun_out/prov_<tag>/c<preset>/{trace,fetch,write,valuclass,valubusy}; tools/make_traffic.py turns
# them into profiles/<tag>/ and profiles/traffic.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${TAG:?set TAG}
presets=${*:-3 2 4 5}
for p in $presets; do
  case $p in
    3) args="--steps 30 --warmup 30 --cpu-seconds 0" ;;
    2) args="--config 2 --steps 50 --warmup 50 --cpu-seconds 0" ;;
    4) args="--config 4 --steps 10 --warmup 5 --cpu-seconds 0" ;;
    5) args="--config 5 --steps 20 --warmup 5 --cpu-seconds 0" ;;
    *) echo "unknown preset $p"; exit 2 ;;
  esac
  out=gpurun_out/prov_$tag/c$p
  mkdir -p $out
  echo "python3 bench.py $args" > $out/args.txt
  echo "[prov] preset $p trace $(date +%T)"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/trace.json 2> $out/trace.err || exit 1
  echo "[prov] preset $p fetch $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py $args > $out/fetch.json 2> $out/fetch.err || exit 1
  echo "[prov] preset $p write $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py $args > $out/write.json 2> $out/write.err || exit 1
  echo "[prov] preset $p valuclass $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES \
    --output-format csv -d $out/valuclass -o run -- python3 bench.py $args > $out/valuclass.json 2> $out/valuclass.err || exit 1
  echo "[prov] preset $p valubusy $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d $out/valubusy -o run -- python3 bench.py $args > $out/valubusy.json 2> $out/valubusy.err || exit 1
done
echo "[prov] done $(date +%T)"
