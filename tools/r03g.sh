set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
timeout -k 10 200 bash tools/cli_trace.sh gpurun_out/r03g/cli || exit 1
for ws in 2 4 8; do
  timeout -k 10 240 python3 tools/c4_rank_share.py --ws $ws > gpurun_out/r03g/c4_rank_share_ws$ws.json 2> gpurun_out/r03g/c4_ws$ws.err || { tail -5 gpurun_out/r03g/c4_ws$ws.err; exit 1; }
done
timeout -k 10 240 python3 tools/c4_rank_share.py --ws 8 --rank 7 > gpurun_out/r03g/c4_rank_share_ws8_rank7.json 2>/dev/null || exit 1
python3 - <<'PY'
import json
for f in ("ws2","ws4","ws8","ws8_rank7"):
    d=json.load(open(f"gpurun_out/r03g/c4_rank_share_{f}.json"))
    print(f, round(d["sketch_shard_ms"],3), round(d["dist_ms"],3), {k[:14]:v["total_ms"] for k,v in d["dist_kernels"].items()})
PY
