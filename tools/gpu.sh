# GPU-box steps, one parametrised script (run through gpurun; every step has its own time limit and
# the first failure ends the call).  Outputs go to gpurun_out/TAG/.
#
#   gpurun --timeout 900 -- 'bash tools/gpu.sh TAG STEP [STEP ...]'
#
# STEPs (run in order):
#   tests        every -m gpu test (the driver's round-end tier)
#   tests:EXPR   the -m gpu tests selected by -k EXPR
#   smoke        __graft_entry__.smoke()
#   bench        the default bench line (C3 headline + C5 + C4 + medium) -> bench.json
#   profile      rocprofv3 kernel trace of a short bench + FETCH / WRITE / VALU PMC passes, summarised
#                into pmc_traffic.json (tools/pmc_summary.py) and kernel_stats.csv
#   pmc_c5       PMC passes over one C5 consensus, per kernel (k_gemm_i8 split into grid / mixed)
#   shard        one 8-GPU C5 shard (125k x 4096) as a one-rank consensus (tools/c5_shard_latency.py)
#   host         the drop-in's host-memory path at C5, copy and in-place `original` (tools/c5_host_latency.py)
#   shard_prof   rocprofv3 kernel trace of the shard run (per-launch times: shard_kt/)
#   dist         the 2-process tests and bench.py as the driver launches N=2 (gloo: both ranks on cuda:0)
#   selfdist     bench.py --gpus 2 with no launcher (bench.py starts the ranks itself; gloo on cuda:0)
#   ab_c3=L1,L2  C3 bench of several libpcx builds (PCX_LIB), alternating twice
#   ab_med=L1,L2 the medium-round (100 x 50) line of several libpcx builds, alternating twice
#   ab_c5=L1,L2  C5 latency of several libpcx builds, alternating twice
#   ab_shard=L1,L2  one C5 shard's latency of several libpcx builds, alternating twice
#   kt_c5=L1,L2  rocprofv3 kernel trace of one C5 consensus per libpcx build, per-kernel times (tools/kt_top.py)
#   i8bench      the int8 covariance GEMM variants at the C5 shapes (tools/i8bench, built on the CPU)
#   i8ks=S:K,..  the product int8 GEMM on shape S (mixed | grid) at each k-slice count K
#   i8pmc=V      SQ / LDS / cache PMC passes over the mixed-block GEMM, reference kernel and variant V
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O

run_tests() {  # $1: log name, rest: pytest args
  local log=$1; shift
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "$@" > $O/$log 2>&1 \
    || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)|Error" $O/$log | head -20; tail -5 $O/$log; exit 11; }
  tail -1 $O/$log
}

c5_line() {  # $1 json (the last line starting with '{': gloo prints its connection notes to stdout), $2 label
  python3 -c "import json,sys; c=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['c5']; s=c['stage_ms']; print('%-24s C5 %.1f ms (mean %.1f) ' % (sys.argv[2], c['latency_ms'], c.get('latency_ms_mean', 0)) + ' '.join('%s %.1f' % (k[2:], v) for k, v in list(s.items())[:10]))" "$1" "$2"
}

for STEP in "$@"; do
  case $STEP in
    tests) run_tests pytest_gpu.log ;;
    tests:*) run_tests pytest_sel.log -k "${STEP#tests:}" ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 12; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 13; }
      python3 -c "import json; d=json.load(open('$O/bench.json')); print('C3', round(d['value']/1e6,2), 'M/s kernel', round(d['roofline']['kernel_ms'],3), 'ms frac', round(d['roofline']['frac'],3), '| C5', round(d['c5']['latency_ms'],1), d['c5'].get('latency_ms_all'), '| C4', round(d['c4']['latency_ms'],2), '| medium', round(d['medium']['rounds_per_s']/1e6,2), 'M/s')"
      c5_line $O/bench.json bench ;;
    profile)
      ARGS="--steps 5 --warmup 1 --no-cpu-baseline --c5-steps 1 --no-c4"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $ARGS > $O/kt.log 2>&1 || { echo "kernel-trace rc=$?"; tail -5 $O/kt.log; exit 14; }
      for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
        timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/$C -o pmc -- python3 bench.py $ARGS > $O/$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -5 $O/$C.log; exit 15; }
      done
      KS=$(find $O/kt -name "kt_kernel_stats.csv" | head -1)
      python3 tools/pmc_summary.py --stats "$KS" --trace "$(find $O/kt -name 'kt_kernel_trace.csv' | head -1)" --fetch "$(find $O/FETCH_SIZE -name 'pmc_counter_collection.csv' | head -1)" \
          --write "$(find $O/WRITE_SIZE -name 'pmc_counter_collection.csv' | head -1)" \
          --valu "$(find $O/SQ_INSTS_VALU -name 'pmc_counter_collection.csv' | head -1)" --out $O/pmc_traffic.json \
          --note "bench.py $ARGS (C3 65536 x 50x20 with every output + one C5 1M x 4k), MI355X" > $O/summary.log 2>&1 || { echo summary failed; tail -5 $O/summary.log; exit 16; }
      cp "$KS" $O/kernel_stats.csv
      echo profile ok ;;
    pmc_c5)
      ARGS="--steps 1 --warmup 0 --rounds 4096 --no-cpu-baseline --no-c4 --c5-steps 1"
      i=0
      for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
               "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
               "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o pmc -- python3 bench.py $ARGS > $O/p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -5 $O/p$i.log; exit 17; }
      done
      python3 tools/pmc_summary.py --per-kernel "$O" > $O/pmc_c5.txt 2>&1 || { echo "pmc summary failed"; tail -5 $O/pmc_c5.txt; exit 18; }
      cat $O/pmc_c5.txt ;;
    shard)
      timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/w8.json 2> $O/w8.err || { echo "shard rc=$?"; tail -20 $O/w8.err; exit 19; }
      python3 -c "import json; d=json.load(open('$O/w8.json')); print('shard', round(d['latency_ms'],2), 'ms;', ' '.join('%s %.2f' % (k[2:], v) for k, v in list(d.get('stage_ms', {}).items())[:10]))" ;;
    host)  # the drop-in's host-memory path at C5: copies in and out + consensus (tools/c5_host_latency.py)
      timeout -k 10 900 python -u tools/c5_host_latency.py 3 > $O/host.json 2> $O/host.err || { echo "host rc=$?"; tail -20 $O/host.err; exit 31; }
      grep '"mode"' $O/host.err ;;
    shard_prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard_kt -o kt -- python3 tools/c5_shard_latency.py 8 3 > $O/shard_kt.log 2>&1 || { echo "shard kernel-trace rc=$?"; tail -5 $O/shard_kt.log; exit 27; }
      KT=$(find $O/shard_kt -name "kt_kernel_trace.csv" | head -1)
      python3 tools/kt_top.py $KT -1 24 && python3 tools/trace_gaps.py $KT -1 15 > $O/shard_gaps.txt && head -12 $O/shard_gaps.txt ;;
    dist)
      timeout -k 10 240 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_dist.log 2>&1 || { echo "pytest dist rc=$?"; tail -40 $O/pytest_dist.log; exit 20; }
      tail -1 $O/pytest_dist.log
      PCX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --c5-steps 2 \
          --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || { echo "bench2 rc=$?"; tail -30 $O/bench2.err; exit 21; }
      c5_line $O/bench2.json "N=2 gloo" ;;
    selfdist)  # bench.py --gpus 2 with NO launcher: it must start the 2 ranks itself (gloo: both on cuda:0)
      PCX_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 --c5-steps 2 \
          --no-cpu-baseline > $O/bench_self2.json 2> $O/bench_self2.err || { echo "selfdist rc=$?"; tail -30 $O/bench_self2.err; exit 30; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['c5']; print('self-launched: n_gpus', d['n_gpus'], 'launcher', d['launcher'], 'devices', [x['device'] for x in d['devices']], '| C5 n_gpus', c['n_gpus'], 'comm', c['comm'], 'ctx_world', c['ctx_world'], 'rccl_world', c['rccl_world'])" $O/bench_self2.json
      c5_line $O/bench_self2.json "N=2 self gloo" ;;
    ab_c3=*)
      IFS=, read -ra LIBS <<< "${STEP#ab_c3=}"
      for i in 1 2; do for L in "${LIBS[@]}"; do
        PCX_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --c5-steps 0 --no-c4 --steps 30 > $O/ab.json 2> $O/ab.err || { echo "ab rc=$? ($L)"; tail -3 $O/ab.err; exit 22; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-36s %.3f ms  %.2fM rounds/s' % (sys.argv[2], d['roofline']['kernel_ms'], d['value']/1e6))" $O/ab.json "$L"
      done; done ;;
    ab_med=*)  # the medium-round (100 x 50) line of several libpcx builds, alternating twice
      IFS=, read -ra LIBS <<< "${STEP#ab_med=}"
      for i in 1 2; do for L in "${LIBS[@]}"; do
        PCX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --c5-steps 0 --steps 5 > $O/abm.json 2> $O/abm.err || { echo "ab_med rc=$? ($L)"; tail -3 $O/abm.err; exit 33; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); m=d['medium']; print('%-28s medium %.3f ms  %.3fM rounds/s' % (sys.argv[2], m['ms'], m['rounds_per_s']/1e6))" $O/abm.json "$L"
      done; done ;;
    ab_c5=*)
      IFS=, read -ra LIBS <<< "${STEP#ab_c5=}"
      for i in 1 2; do for L in "${LIBS[@]}"; do
        PCX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4 --c5-steps 3 --steps 3 > $O/ab.json 2> $O/ab.err || { echo "ab rc=$? ($L)"; tail -3 $O/ab.err; exit 23; }
        c5_line $O/ab.json "$L"
      done; done ;;
    kt_c5=*)
      IFS=, read -ra LIBS <<< "${STEP#kt_c5=}"
      i=0
      for L in "${LIBS[@]}"; do
        i=$((i+1))
        PCX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt$i -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c5-steps 1 --no-c4 > $O/kt$i.log 2>&1 || { echo "kt_c5 rc=$? ($L)"; tail -5 $O/kt$i.log; exit 30; }
        echo "== $L"
        python3 tools/kt_top.py $(find $O/kt$i -name "kt_kernel_trace.csv" | head -1) -1 ${KT_TOP:-14} ${KT_LAUNCHES:-k_sel_hist} || exit 31
      done ;;
    ab_shard=*)
      IFS=, read -ra LIBS <<< "${STEP#ab_shard=}"
      for i in 1 2; do for L in "${LIBS[@]}"; do
        PCX_LIB=$L timeout -k 10 200 python -u tools/c5_shard_latency.py 8 5 > $O/abs.json 2> $O/abs.err || { echo "ab_shard rc=$? ($L)"; tail -3 $O/abs.err; exit 28; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-24s shard %.2f ms; ' % (sys.argv[2], d['latency_ms']) + ' '.join('%s %.2f' % (k[2:], v) for k, v in list(d.get('stage_ms', {}).items())[:10]))" $O/abs.json "$L"
      done; done ;;
    ab_host=*)  # the host-memory path's latency (tools/c5_host_latency.py) of several libpcx builds
      IFS=, read -ra LIBS <<< "${STEP#ab_host=}"
      for L in "${LIBS[@]}"; do
        PCX_LIB=$L timeout -k 10 300 python -u tools/c5_host_latency.py 2 > $O/abh.json 2> $O/abh.err || { echo "ab_host rc=$? ($L)"; tail -5 $O/abh.err; exit 32; }
        echo "== $L"; grep '"mode"' $O/abh.err | cut -c1-220
      done ;;
    i8bench)
      timeout -k 10 300 tools/i8bench/i8bench 5 > $O/i8bench.txt 2>&1 || { echo "i8bench rc=$?"; tail -20 $O/i8bench.txt; exit 24; }
      cat $O/i8bench.txt ;;
    i8ks=*)  # i8ks=SHAPE:K1,K2,...  the product kernel at each k-slice count (SHAPE: mixed | grid)
      A=${STEP#i8ks=}
      timeout -k 10 300 tools/i8bench/i8bench 3 1000064 product "${A%%:*}" "${A#*:}" > $O/i8ks_${A%%:*}.txt 2>&1 || { echo "i8ks rc=$?"; tail -20 $O/i8ks_${A%%:*}.txt; exit 29; }
      grep -v "small check" $O/i8ks_${A%%:*}.txt ;;
    i8pmc=*)  # i8pmc=V or i8pmc=V:SHAPE (SHAPE: mixed (default) | grid | gg)
      V=${STEP#i8pmc=}
      SH=mixed
      case $V in *:*) SH=${V#*:}; V=${V%%:*} ;; esac
      i=0
      for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
               "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
               "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/i8p$i -o pmc -- tools/i8bench/i8bench 2 1000064 "$V" $SH > $O/i8p$i.log 2>&1 || { echo "i8pmc pass $i rc=$?"; tail -5 $O/i8p$i.log; exit 25; }
      done
      python3 tools/pmc_summary.py --per-kernel "$O" --glob "i8p*" > $O/i8pmc.txt 2>&1 || { echo "i8pmc summary failed"; tail -5 $O/i8pmc.txt; exit 26; }
      cat $O/i8pmc.txt ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
