set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s11
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k prefilled --timeout 120 --timeout-method thread > gpurun_out/r03s11/pytest.log 2>&1 || { tail -40 gpurun_out/r03s11/pytest.log; exit 1; }
tail -1 gpurun_out/r03s11/pytest.log
FPM_C4_PREFILL=0.1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3 --no-c5 --no-cli --no-fp-text --no-split > gpurun_out/r03s11/c4p.json 2> gpurun_out/r03s11/c4p.err || { tail -20 gpurun_out/r03s11/c4p.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r03s11/c4p.json').read().strip().splitlines()[-1]); print('c4 prefill 0.1', d['c4_dist']['ms_per_step'], d['c4_dist']['parity'], d['parity']['all_ok'])"
AB_LEG=c4 timeout -k 10 900 bash tools/env_ab.sh FPM_C4_PREFILL=0.05 FPM_C4_PREFILL=0.1 FPM_C4_PREFILL=0.15 > gpurun_out/r03s11/env.txt 2>&1 || { tail -5 gpurun_out/r03s11/env.txt; exit 1; }
cat gpurun_out/r03s11/env.txt
