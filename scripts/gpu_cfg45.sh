set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload cfg4 --steps 5 --warmup 1 > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err; rc=$?
echo "cfg4 rc=$rc"; cat gpurun_out/cfg4.json; tail -3 gpurun_out/cfg4.err
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload cfg5 --pairs 100000 --steps 2 --warmup 1 --check-all > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err; rc=$?
echo "cfg5 rc=$rc"; cat gpurun_out/cfg5.json; tail -3 gpurun_out/cfg5.err
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload cfg5 --pairs 100000 --gap-open -2 --steps 2 --warmup 1 --check-all > gpurun_out/cfg5a.json 2> gpurun_out/cfg5a.err; rc=$?
echo "cfg5a rc=$rc"; cat gpurun_out/cfg5a.json; tail -3 gpurun_out/cfg5a.err
