#!/bin/bash
# Build libfdcn.so from the csrc/ + include/ of a git revision (or the working
# tree for "WT") into ab/TAG/libfdcn.so, for A/B timing through bench.py --lib
# (capi.LIB_PATH).  KREV (optional): take fdcn_kernels.hip alone from that
# revision, everything else from REV -- a kernel A/B on the current ABI.
# ABFLAGS (environment): extra hipcc flags, e.g. -DFDCN_STAMPS for a diagnostic build;
# KSRC: a kernel source file to use in place of fdcn_kernels.hip.
# Usage: bash tools/build_ab.sh TAG [REV] [KREV]
set -euo pipefail
TAG=$1; REV=${2:-WT}; KREV=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$(mktemp -d)
mkdir -p "$SRC/finite_difference_amd/csrc" "$SRC/include" "$ROOT/ab/$TAG"
if [ "$REV" = "WT" ]; then
  cp "$ROOT"/finite_difference_amd/csrc/*.hip "$ROOT"/finite_difference_amd/csrc/*.h "$SRC/finite_difference_amd/csrc/"
  cp "$ROOT"/include/*.h "$SRC/include/"
else
  for f in $(git -C "$ROOT" ls-tree --name-only "$REV" finite_difference_amd/csrc/ include/); do
    git -C "$ROOT" show "$REV:$f" > "$SRC/$f"
  done
fi
if [ -n "${KSRC:-}" ]; then  # an edited kernel source (diagnostic A/B builds)
  cp "$KSRC" "$SRC/finite_difference_amd/csrc/fdcn_kernels.hip"
elif [ -n "$KREV" ]; then
  git -C "$ROOT" show "$KREV:finite_difference_amd/csrc/fdcn_kernels.hip" \
      > "$SRC/finite_difference_amd/csrc/fdcn_kernels.hip"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared ${ABFLAGS:-} \
    -o "$ROOT/ab/$TAG/libfdcn.so" "$SRC"/finite_difference_amd/csrc/*.hip
rm -rf "$SRC"
echo "$ROOT/ab/$TAG/libfdcn.so"
