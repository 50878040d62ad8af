#!/bin/bash
# tools/build_variant.sh NAME "EXTRA_HIPFLAGS" [GIT_REV] — build fp-mash_amd/lib/libfpmash_NAME.so
# beside the product for same-box A/B runs (tools/knobs_ab.sh NAME ...): the current kernel
# sources with extra compile-time knobs, or (GIT_REV) the csrc/ tree of an earlier commit.
set -euo pipefail
NAME=${1:?name}; FLAGS=${2:-}; REV=${3:-}
cd "$(dirname "$0")/../fp-mash_amd"
SRC=csrc
if [ -n "$REV" ]; then
  T=$(mktemp -d); SRC=$T/a/b/csrc; mkdir -p "$SRC" "$T/a/include"
  git show "$REV:include/fpmash.h" > "$T/a/include/fpmash.h"
  for f in $(git ls-tree --name-only "$REV" csrc/); do git show "$REV:fp-mash_amd/$f" > "$SRC/$(basename "$f")"; done
fi
OUT=build/variant_$NAME; mkdir -p "$OUT" lib
HIPCC=/opt/rocm/bin/hipcc
HF="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -I../include $FLAGS"
pids=()
for k in sketch fingerprint dist dist_index seqparse; do
  src="$SRC/$k.hip"
  # KSRC_<name>=path swaps one kernel source (e.g. an older dist.hip beside the current API)
  ov="KSRC_$k"; [ -n "${!ov:-}" ] && src="${!ov}"
  $HIPCC $HF -I"$PWD/csrc" -c "$src" -o "$OUT/$k.o" & pids+=($!)
done
for c in "$SRC"/*.cpp; do
  $HIPCC $HF -c "$c" -o "$OUT/$(basename "$c" .cpp).o" & pids+=($!)
done
id=$(cat "$SRC"/*.hip "$SRC"/*.cpp "$SRC"/*.hpp | sha256sum | cut -c1-16)
printf 'extern "C" const char *fpm_build_id(void) { return "%s"; }\nextern "C" const char fpm_build_id_tag[] = "fpm-build-id:%s";\n' $id $id > "$OUT/build_id.cpp"
$HIPCC $HF -c "$OUT/build_id.cpp" -o "$OUT/build_id.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "lib/libfpmash_$NAME.so" "$OUT"/*.o -ldl
echo "lib/libfpmash_$NAME.so"
