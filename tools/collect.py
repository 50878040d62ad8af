#!/usr/bin/env python3
"""tools/collect.py TAG ROUND — copy one GPU call's evidence (gpurun_out/TAG/, written by
tools/round.sh on the box) into profiles/ROUND/ in the build container:

  pmc_traffic.json, pmc_c3/c4/c5.json  -> profiles/ROUND/ (the names bench.py reads)
  kernel_stats.csv                     -> profiles/ROUND/kernel_stats_TAG.csv
  bench.json, bench_detail.json        -> profiles/ROUND/bench_TAG.json, bench_detail_TAG.json
  pytest.log                           -> profiles/ROUND/gpu_tests_TAG.txt
  rehearse_n*.json                     -> profiles/ROUND/rehearse_n*_TAG.json

Every counter file and the kernel stats carry the build id of the libfpmash.so they measured;
a file whose id differs from the local build's is refused (the bench would not attach it)
unless --force."""
import argparse
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fp-mash_amd"))
import fpmash  # noqa: E402


def file_build_id(path):
    if path.endswith(".json"):
        return json.load(open(path)).get("build_id")
    with open(path) as f:
        first = f.readline()
    return first.split("fpm_build_id=")[1].split()[0] if "fpm_build_id=" in first else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("round")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles", a.round)
    os.makedirs(dst, exist_ok=True)
    want = fpmash.build_id()
    plan = [(f"pmc_{x}.json", f"pmc_{x}.json", True) for x in ("traffic", "c3", "c4", "c5")]
    plan += [("kernel_stats.csv", f"kernel_stats_{a.tag}.csv", True),
             ("bench.json", f"bench_{a.tag}.json", False),
             ("bench_detail.json", f"bench_detail_{a.tag}.json", False),
             ("pytest.log", f"gpu_tests_{a.tag}.txt", False),
             ("rehearse_n2.json", f"rehearse_n2_{a.tag}.json", False),
             ("rehearse_n4.json", f"rehearse_n4_{a.tag}.json", False)]
    bad = 0
    for name, out, stamped in plan:
        p = os.path.join(src, name)
        if not os.path.exists(p):
            continue
        if stamped:
            have = file_build_id(p)
            if have != want and not a.force:
                print(f"REFUSED {name}: build {have}, local libfpmash.so is {want}")
                bad += 1
                continue
        shutil.copyfile(p, os.path.join(dst, out))
        print(f"{name} -> profiles/{a.round}/{out}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
