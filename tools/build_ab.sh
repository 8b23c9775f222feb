#!/bin/bash
# Build libfdcn.so from the csrc/ + include/ of a git revision (or the working
# tree for "WT") into ab/TAG/libfdcn.so, for A/B timing through bench.py --lib
# (capi.LIB_PATH).  KREV (optional): take fdcn_kernels.hip alone from that
# revision, everything else from REV -- a kernel A/B on the current ABI.
# ABFLAGS (environment): extra hipcc flags, e.g. -DFDCN_STAMPS for a diagnostic build;
# KSRC: a kernel source file to use in place of fdcn_kernels.hip.
#
# Provenance (round 6): next to the library, ab/TAG/PROVENANCE.txt records
# what was compiled -- HEAD, the revision arguments, the flags, the sha256 of
# every source file that went into the build, and `git diff HEAD` of csrc/ and
# include/ for a working-tree build -- and ab/TAG/src/ keeps the sources
# themselves.  A run that faults can then be traced to its exact source
# (tools/gpu_ab.sh copies the record under profiles/ when a run fails).
# Usage: bash tools/build_ab.sh TAG [REV] [KREV]
set -euo pipefail
TAG=$1; REV=${2:-WT}; KREV=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$(mktemp -d)
OUT="$ROOT/ab/$TAG"
mkdir -p "$SRC/finite_difference_amd/csrc" "$SRC/include" "$OUT"
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
    -o "$OUT/libfdcn.so" "$SRC"/finite_difference_amd/csrc/*.hip
{
  echo "tag: $TAG"
  echo "built: $(date -u +%Y-%m-%dT%H:%M:%SZ)"
  echo "head: $(git -C "$ROOT" rev-parse HEAD)"
  echo "rev: $REV"
  echo "krev: ${KREV:-}"
  echo "ksrc: ${KSRC:-}"
  echo "abflags: ${ABFLAGS:-}"
  echo "sha256 (sources compiled):"
  (cd "$SRC" && sha256sum finite_difference_amd/csrc/* include/*)
  echo "libfdcn.so: $(sha256sum "$OUT/libfdcn.so" | cut -d' ' -f1)"
  if [ "$REV" = "WT" ]; then
    echo "git diff HEAD -- finite_difference_amd/csrc include:"
    git -C "$ROOT" diff HEAD -- finite_difference_amd/csrc include
    for f in $(git -C "$ROOT" ls-files --others --exclude-standard finite_difference_amd/csrc include); do
      echo "untracked: $f"
    done
  fi
} > "$OUT/PROVENANCE.txt"
rm -rf "$OUT/src"
mv "$SRC" "$OUT/src"
echo "$OUT/libfdcn.so"
