set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k
for i in 1 2 3 4 5; do
  for m in serial parallel nosecond; do
    timeout -k 5 30 tools/micro/init_par $m >> gpurun_out/r03k/init_par.txt || exit 1
  done
done
sort gpurun_out/r03k/init_par.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multirank.py tests/test_cli.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03k/pytest.log 2>&1 || { tail -30 gpurun_out/r03k/pytest.log; exit 1; }
tail -1 gpurun_out/r03k/pytest.log
OUT=gpurun_out/r03k/cli REPS=5 timeout -k 10 300 bash tools/cli_ab.sh HSA_ENABLE_SDMA=0 || exit 1
for ws in 2 8; do
  timeout -k 10 240 python3 tools/c4_rank_share.py --ws $ws > gpurun_out/r03k/c4_rank_share_ws$ws.json 2> gpurun_out/r03k/c4_ws$ws.err || { tail -5 gpurun_out/r03k/c4_ws$ws.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ("ws2","ws8"):
    d=json.load(open(f"gpurun_out/r03k/c4_rank_share_{f}.json"))
    print(f, round(d["sketch_shard_ms"],3), round(d["dist_ms"],3), {k[:14]:v["total_ms"] for k,v in d["dist_kernels"].items()})
PY
