#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer build of the HOST code of libwam_hip.so with the
# plan fuzz driver (tests/native/plan_fuzz.cpp). Host-only compilation (--offload-host-only): no
# device code is built, nothing runs on a GPU; the sanitizers go on the host side only (each
# -fsanitize= after -Xarch_host). Output: build/sanitize/plan_fuzz (git-ignored).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/build/sanitize
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all)
FLAGS=(--offload-host-only -O1 -g -fno-omit-frame-pointer -std=c++17 -fPIC -Wno-unused-function)
objs=()
pids=()
for s in "$ROOT"/wam_amd/csrc/*.hip; do
  o=$OUT/$(basename "$s" .hip).o
  objs+=("$o")
  "$HIPCC" -x hip "${FLAGS[@]}" "${SAN[@]}" -c "$s" -o "$o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" -x hip "${FLAGS[@]}" "${SAN[@]}" -c "$ROOT/tests/native/plan_fuzz.cpp" -o "$OUT/plan_fuzz.o"
# host-only objects still reference their (absent) device code blobs: zero-filled stand-ins satisfy
# the linker; nothing is ever launched from this binary
nm "${objs[@]}" "$OUT/plan_fuzz.o" 2>/dev/null | awk '/ U __hip_fatbin_/{print $2}' | sort -u |
  awk '{print "char " $1 "[4096] __attribute__((aligned(4096)));"}' > "$OUT/fatbin_stubs.c"
gcc -c "$OUT/fatbin_stubs.c" -o "$OUT/fatbin_stubs.o"
"$HIPCC" "${SAN[@]}" -o "$OUT/plan_fuzz" "$OUT/plan_fuzz.o" "${objs[@]}" "$OUT/fatbin_stubs.o"
echo "$OUT/plan_fuzz"
