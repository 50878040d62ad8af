set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03r
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03r/pytest.log 2>&1 || { tail -30 gpurun_out/r03r/pytest.log; exit 1; }
tail -1 gpurun_out/r03r/pytest.log
timeout -k 10 700 bash tools/ab_bench.sh fp-mash_amd/lib_ab/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 > gpurun_out/r03r/ab.txt 2>&1 || { tail -5 gpurun_out/r03r/ab.txt; exit 1; }
cat gpurun_out/r03r/ab.txt
for g in 0 2048 8192 32768; do
  FPM_FILL_GRID=$g timeout -k 10 240 python3 tools/c4_rank_share.py --ws 8 > gpurun_out/r03r/ws8_grid$g.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r03r/ws8_grid$g.json'))
print('grid $g', round(d['dist_ms'],3), {k[:14]:v['total_ms'] for k,v in d['dist_kernels'].items()})"
done
