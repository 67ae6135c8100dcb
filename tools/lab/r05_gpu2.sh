# Round 5, call 2: the service re-arm fix and the XXH64 single-launch
# descriptor kernel on hardware.  Service tests (12 s soak included), the
# descriptor / XXH64 parity tests, the default bench line (sweep, config 1
# with the all-cores in-memory leg), then a 60 s soak.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_service.py > $O/service_tests.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "desc or xxh64 or first_bad or shape" tests/ > $O/desc_tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 150 tests/cpp/service_threads_test --soak 60 > $O/soak60.txt 2>&1
rc=$?
echo "exit $rc"
grep -E "PASS|FAIL|ERROR" $O/service_tests.log | tail -40; tail -3 $O/service_tests.log; tail -3 $O/desc_tests.log
python3 -c "
import json,sys
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'checks', d.get('checks_all_ranks_pass'))
for e in d.get('sweep', []): print(e.get('key'), e.get('avg_launch_ms'), e.get('frac'), e.get('parity',{}).get('mismatches'), e.get('corruption_drill',{}).get('pass'))
for k in ('cpu_baseline','cpu_ref_inmem','cpu_all_cores','cpu_ref_inmem_all_cores'): print(k, (d.get(k) or {}).get('value'), (d.get(k) or {}).get('cores'))
" || true
cat $O/soak60.txt
exit $rc
