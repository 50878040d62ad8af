set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03x/pytest.log 2>&1 || { tail -40 gpurun_out/r03x/pytest.log; exit 1; }
tail -1 gpurun_out/r03x/pytest.log
timeout -k 10 600 bash tools/env_ab.sh FPM_FILL_ROWS=1 > gpurun_out/r03x/env_c2.txt 2>&1 || { tail -5 gpurun_out/r03x/env_c2.txt; exit 1; }
cat gpurun_out/r03x/env_c2.txt
AB_LEG=c4 timeout -k 10 600 bash tools/env_ab.sh FPM_FILL_ROWS=1 > gpurun_out/r03x/env_c4.txt 2>&1 || { tail -5 gpurun_out/r03x/env_c4.txt; exit 1; }
cat gpurun_out/r03x/env_c4.txt
for a in "2 0" "4 0" "8 0" "8 7"; do
  set -- $a
  timeout -k 10 240 python3 tools/c4_rank_share.py --ws $1 --rank $2 > gpurun_out/r03x/c4_rank_share_ws$1_rank$2.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r03x/c4_rank_share_ws$1_rank$2.json'))
print('ws $1 rank $2', round(d['rank_step_ms_excl_gather'],3), round(d['dist_ms'],3), {k[:14]:v['total_ms'] for k,v in d['dist_kernels'].items()})"
done
