#!/bin/bash
# tools/r05_final_ab.sh TAG LIB_B — the round-5 evidence pass (tools/r05_final.sh TAG), then a
# same-box A/B of the current build (A) against LIB_B on the C2 step and the C4 leg.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r05_final.sh "$1" && \
bash tools/lib_ab_c2.sh fp-mash_amd/lib/libfpmash.so "$2" 2 && \
bash tools/lib_ab_leg.sh c4 fp-mash_amd/lib/libfpmash.so "$2" 2
