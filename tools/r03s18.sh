set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s18
FPM_SEL_OVERLAP=1 timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3 --no-c4 --no-cli --no-fp-text --no-split > gpurun_out/r03s18/c5.json 2> gpurun_out/r03s18/c5.err || { tail -20 gpurun_out/r03s18/c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r03s18/c5.json').read().strip().splitlines()[-1]); c=d['c5_sketch']; print('overlap c5', c['ms_per_step'], c['parity'], d['parity']['all_ok'])"
AB_LEG=c5 timeout -k 10 900 bash tools/env_ab.sh FPM_SEL_OVERLAP=1 > gpurun_out/r03s18/env.txt 2>&1 || { tail -5 gpurun_out/r03s18/env.txt; exit 1; }
cat gpurun_out/r03s18/env.txt
