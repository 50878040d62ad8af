set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03b/pytest.log 2>&1 || { tail -30 gpurun_out/r03b/pytest.log; exit 1; }
tail -2 gpurun_out/r03b/pytest.log
timeout -k 10 120 python tools/micro/fp_stall.py > gpurun_out/r03b/fp_stall.log 2>&1 || { tail -20 gpurun_out/r03b/fp_stall.log; exit 1; }
cat gpurun_out/r03b/fp_stall.log
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r03b/fptrace -o fp --output-format csv -- python3 tools/micro/fp_stall.py > gpurun_out/r03b/fp_stall_prof.log 2>&1 || { tail -20 gpurun_out/r03b/fp_stall_prof.log; exit 1; }
for ws in 2 4 8; do
  timeout -k 10 240 python tools/c4_rank_share.py --ws $ws --rank 0 > gpurun_out/r03b/c4_share_ws$ws.json 2> gpurun_out/r03b/c4_share_ws$ws.err || { tail -20 gpurun_out/r03b/c4_share_ws$ws.err; exit 1; }
  cut -c1-900 gpurun_out/r03b/c4_share_ws$ws.json
done
timeout -k 10 240 python tools/c4_rank_share.py --ws 8 --rank 7 > gpurun_out/r03b/c4_share_ws8_r7.json 2> gpurun_out/r03b/c4_share_ws8_r7.err || { tail -20 gpurun_out/r03b/c4_share_ws8_r7.err; exit 1; }
cut -c1-900 gpurun_out/r03b/c4_share_ws8_r7.json
timeout -k 10 400 bash tools/env_ab.sh FPM_IDX_ONEPASS=0 > gpurun_out/r03b/env_ab_c2.txt 2>&1 || { tail -20 gpurun_out/r03b/env_ab_c2.txt; exit 1; }
cat gpurun_out/r03b/env_ab_c2.txt
AB_LEG=c4 timeout -k 10 600 bash tools/env_ab.sh FPM_IDX_ONEPASS=0 > gpurun_out/r03b/env_ab_c4.txt 2>&1 || { tail -20 gpurun_out/r03b/env_ab_c4.txt; exit 1; }
cat gpurun_out/r03b/env_ab_c4.txt
FPMASH_LIB=$PWD/fp-mash_amd/lib/libfpmash_keq.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "dist or refset" --timeout 120 --timeout-method thread > gpurun_out/r03b/pytest_keq.log 2>&1 || { tail -30 gpurun_out/r03b/pytest_keq.log; exit 1; }
tail -1 gpurun_out/r03b/pytest_keq.log
timeout -k 10 500 bash tools/knobs_ab.sh base keq lay1 keqlay1 > gpurun_out/r03b/knobs_rank.txt 2>&1 || { tail -20 gpurun_out/r03b/knobs_rank.txt; exit 1; }
cat gpurun_out/r03b/knobs_rank.txt
