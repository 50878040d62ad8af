set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s14
V=$PWD/fp-mash_amd/lib/libfpmash_cmp64.so
FPMASH_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py tests/test_gpu_seqparse.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03s14/pytest.log 2>&1 || { tail -40 gpurun_out/r03s14/pytest.log; exit 1; }
tail -1 gpurun_out/r03s14/pytest.log
timeout -k 10 600 bash tools/knobs_ab.sh base cmp64 > gpurun_out/r03s14/c2.txt 2>&1 || { tail -5 gpurun_out/r03s14/c2.txt; exit 1; }
cat gpurun_out/r03s14/c2.txt
for i in 1 2; do for n in base cmp64; do
  L=$PWD/fp-mash_amd/lib/libfpmash_$n.so; [ $n = base ] && L=$PWD/fp-mash_amd/lib/libfpmash.so
  FPMASH_LIB=$L timeout -k 10 300 python tools/leg_run.py --leg c5 > gpurun_out/r03s14/c5_$n$i.json 2>&1 || { tail -5 gpurun_out/r03s14/c5_$n$i.json; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r03s14/c5_$n$i.json').read().strip().splitlines()[-1])
print('$n c5', round(d['ms_per_step'],3), {k: round(v['ms'],3) for k, v in d['rank0']['kernels'].items()}, d.get('parity', {}).get('ok'))"
done; done
