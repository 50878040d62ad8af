set -o pipefail
cd /root/repo
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 3 > $O/c2ab.txt 2>&1 || { tail -20 $O/c2ab.txt; exit 1; }
cat $O/c2ab.txt
timeout -k 10 300 bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash_nospec.so fp-mash_amd/lib/libfpmash.so 2 > $O/c2ab_spec.txt 2>&1 || { tail -20 $O/c2ab_spec.txt; exit 1; }
cat $O/c2ab_spec.txt
timeout -k 10 600 bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash_base.so fp-mash_amd/lib/libfpmash.so 2 > $O/c4ab.txt 2>&1 || { tail -20 $O/c4ab.txt; exit 1; }
cat $O/c4ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "dist or index or refset or rank or probe or c4 or mirror or vblocks or cli or speculated or covered" > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /root/repo
O=gpurun_out/r06c
export TMPDIR=/tmp
C2ONLY="--no-cpu-baseline --no-fp-text --no-c3 --no-c4 --no-c5 --no-cli --no-cli-fp --no-split --no-parity --no-full-grid --no-gather-check"
for L in libfpmash libfpmash_nospec; do
  FPMASH_LIB=fp-mash_amd/lib/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$L -o tl -- python3 bench.py $C2ONLY --steps 10 --warmup 3 --detail $O/tl_$L.json > $O/tl_$L.log 2>&1 || { tail -20 $O/tl_$L.log; exit 1; }
  python3 tools/timeline.py $O/tl_$L > $O/timeline_$L.txt; cat $O/timeline_$L.txt; rm -rf $O/tl_$L
done
