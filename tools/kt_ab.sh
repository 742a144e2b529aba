set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m; mkdir -p $O
for L in ${KT_LIBS:-head lfp1}; do
  PCX_LIB=ab/$L/libpcx.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$L -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c5-steps 1 --no-c4 > $O/kt_$L.log 2>&1 || { echo "kt $L rc=$?"; tail -5 $O/kt_$L.log; exit 1; }
done
echo ok
