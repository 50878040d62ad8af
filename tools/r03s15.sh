set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s15
for i in 1 2; do for cfg in "base 0.6" "cmp64 0.6" "cmp64 0.5" "cmp64 0.45" "base 0" "cmp64 0"; do
  set -- $cfg
  L=$PWD/fp-mash_amd/lib/libfpmash_$1.so; [ $1 = base ] && L=$PWD/fp-mash_amd/lib/libfpmash.so
  FPMASH_LIB=$L FPM_BENCH_PREFILL=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-c4 --no-c5 --no-cli --no-fp-text --no-split --no-parity > gpurun_out/r03s15/r_$1_$2_$i.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/r03s15/r_$1_$2_$i.json').read().strip().splitlines()[-1])
print('$1 f=$2', round(d['ms_per_step'],4), {k[:12]:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
done; done
