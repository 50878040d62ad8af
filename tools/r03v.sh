set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py tests/test_cli.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03v/pytest.log 2>&1 || { tail -40 gpurun_out/r03v/pytest.log; exit 1; }
tail -1 gpurun_out/r03v/pytest.log
for rep in 1 2; do
for a in "2 0 0" "2 0 1" "8 0 0" "8 0 1" "4 0 0" "8 7 0"; do
  set -- $a
  FPM_PROBE_COUNT=$3 timeout -k 10 240 python3 tools/c4_rank_share.py --ws $1 --rank $2 > gpurun_out/r03v/c4_rank_share_ws$1_rank$2_c$3.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r03v/c4_rank_share_ws$1_rank$2_c$3.json'))
print('ws $1 rank $2 count $3', round(d['rank_step_ms_excl_gather'],3), round(d['dist_ms'],3), {k[:14]:v['total_ms'] for k,v in d['dist_kernels'].items()})"
done
done
for i in 1 2; do timeout -k 5 60 tools/micro/fill_real; done
