set -o pipefail
cd /root/repo
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
C2ONLY="--no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check"
for L in libfpmash libfpmash_nospec; do
  FPMASH_LIB=fp-mash_amd/lib/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$L -o tl -- python3 bench.py $C2ONLY --steps 10 --warmup 3 --detail $O/tl_$L.json > $O/tl_$L.log 2>&1 || { tail -20 $O/tl_$L.log; exit 1; }
  python3 tools/timeline.py $O/tl_$L > $O/timeline_$L.txt; cat $O/timeline_$L.txt; rm -rf $O/tl_$L
done
