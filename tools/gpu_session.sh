# One GPU-box session of selected steps (run via gpurun from the repo root):
#   bash tools/gpu_session.sh <tag> step [step ...]
# steps:
#   tests            python -m pytest tests -m gpu (log: gpurun_out/<tag>/pytest.log)
#   tests:<expr>     the same restricted with -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench[:args]     python bench.py <args>  (one JSON line -> bench_<n>.json)
#   ubench           tools/ubench/f64_latency (prebuilt in-tree)
#   valumix          tools/ubench/valu_mix (prebuilt): VALU cycles per SIMD by class and waves per SIMD
#   valuclass[:args] / valubusy[:args]   VALU class-count and VALU-busy counter passes over bench.py
#   sq[:args]        SQ counter pass over bench.py <args> (per-kernel CSV)
#   sqmem[:args]     memory-pipeline counter pass over bench.py <args>
#   trace[:args]     rocprofv3 --kernel-trace --stats over bench.py <args>
#   fetch[:args] / write[:args]   FETCH_SIZE / WRITE_SIZE passes
#   py:<file>        python <file> (a tools/ script)
#   env:<K=V>        export K=V for the following steps (A/B knobs such as NNGP_PAIRB_BLOCKS)
# Every GPU step has its own time limit; the first failing step ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
n=0
for step in "$@"; do
  n=$((n+1))
  name=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  echo "== step $n: $step ($(date +%T))"
  case $name in
    tests)
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > $out/pytest_$n.log 2>&1 || { tail -30 $out/pytest_$n.log; exit 1; }
      tail -3 $out/pytest_$n.log ;;
    smoke)
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke_$n.log 2>&1 || { cat $out/smoke_$n.log; exit 1; }
      tail -1 $out/smoke_$n.log ;;
    bench)
      timeout -k 10 300 python -u bench.py $arg > $out/bench_$n.json 2> $out/bench_$n.err || { tail -20 $out/bench_$n.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$out/bench_$n.json')); print('value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'])" ;;
    ubench)
      timeout -k 10 120 tools/ubench/f64_latency > $out/f64_latency.txt 2>&1 || exit 1
      cat $out/f64_latency.txt ;;
    sq)
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES \
        --output-format csv -d $out/sq_$n -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 $arg > $out/sq_$n.json 2> $out/sq_$n.err || { tail -5 $out/sq_$n.err; exit 1; }
      python3 tools/pmc_summary.py $out/sq_$n ;;
    sqmem)
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT \
        --output-format csv -d $out/sqmem_$n -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 $arg > $out/sqmem_$n.json 2> $out/sqmem_$n.err || { tail -5 $out/sqmem_$n.err; exit 1; }
      python3 tools/pmc_summary.py $out/sqmem_$n ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$n -o run -- python3 bench.py --cpu-seconds 0 $arg > $out/trace_$n.json 2> $out/trace_$n.err || { tail -5 $out/trace_$n.err; exit 1; }
      python3 tools/pmc_summary.py $out/trace_$n ;;
    valuclass)
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES \
        --output-format csv -d $out/valuclass_$n -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 $arg > $out/valuclass_$n.json 2> $out/valuclass_$n.err || { tail -5 $out/valuclass_$n.err; exit 1; }
      python3 tools/pmc_summary.py $out/valuclass_$n ;;
    valubusy)
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
        --output-format csv -d $out/valubusy_$n -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 $arg > $out/valubusy_$n.json 2> $out/valubusy_$n.err || { tail -5 $out/valubusy_$n.err; exit 1; }
      python3 tools/pmc_summary.py $out/valubusy_$n ;;
    valumix)
      timeout -k 10 120 tools/ubench/valu_mix > $out/valu_mix.txt 2>&1 || exit 1
      cat $out/valu_mix.txt ;;
    fetch)
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch_$n -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 $arg > $out/fetch_$n.json 2> $out/fetch_$n.err || exit 1
      python3 tools/pmc_summary.py $out/fetch_$n ;;
    write)
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write_$n -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 $arg > $out/write_$n.json 2> $out/write_$n.err || exit 1
      python3 tools/pmc_summary.py $out/write_$n ;;
    env)
      export "$arg"; echo "export $arg" ;;
    counters)
      timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
      wc -l $out/counters.txt ;;
    py)
      timeout -k 10 600 python3 -u $arg > $out/py_$n.log 2>&1 || { tail -20 $out/py_$n.log; exit 1; }
      tail -20 $out/py_$n.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
