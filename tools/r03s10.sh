set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s10
timeout -k 10 400 python -u -m pytest tests/test_multirank.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03s10/pytest.log 2>&1 || { tail -40 gpurun_out/r03s10/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03s10/pytest.log | tail -8
FPM_RANK_PARTS=4 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-cli --no-fp-text --no-split > gpurun_out/r03s10/parts4.json 2> gpurun_out/r03s10/parts4.err || { tail -20 gpurun_out/r03s10/parts4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r03s10/parts4.json').read().strip().splitlines()[-1]); print('parts4', d['ms_per_step'], d['parity']['c2']['ok'], d['parity']['all_ok'])"
