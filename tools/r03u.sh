set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03u
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03u/pytest.log 2>&1 || { tail -40 gpurun_out/r03u/pytest.log; exit 1; }
tail -1 gpurun_out/r03u/pytest.log
for a in "2 0" "4 0" "8 0" "8 7"; do
  set -- $a
  timeout -k 10 240 python3 tools/c4_rank_share.py --ws $1 --rank $2 > gpurun_out/r03u/c4_rank_share_ws$1_rank$2.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r03u/c4_rank_share_ws$1_rank$2.json'))
print('ws $1 rank $2', round(d['rank_step_ms_excl_gather'],3), round(d['dist_ms'],3), {k[:14]:v['total_ms'] for k,v in d['dist_kernels'].items()})"
done
FPM_PROBE_COUNT=1 timeout -k 10 240 python3 tools/c4_rank_share.py --ws 8 > gpurun_out/r03u/ws8_count.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r03u/ws8_count.json'))
print('ws8 FPM_PROBE_COUNT=1', round(d['rank_step_ms_excl_gather'],3), round(d['dist_ms'],3))"
