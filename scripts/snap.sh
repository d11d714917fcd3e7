#!/bin/bash
# Freeze HEAD plus its built libraries into .snap/ (git-ignored) for one gpurun call, so that the working tree can
# change while the call waits for a box:
#   bash scripts/snap.sh && gpurun -- 'bash .snap/scripts/snap_run.sh <tag> <steps...>'
# The libraries must have been built from HEAD's sources (make -C nusiprop_amd/csrc, oracle, tests/hostcheck).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
if ! git diff --quiet HEAD -- nusiprop_amd oracle tests bench.py __graft_entry__.py scripts include; then
  echo "snap: uncommitted changes in the sources; commit first" >&2
  exit 1
fi
rm -rf .snap
mkdir .snap
git archive HEAD | tar -x -C .snap
rm -rf .snap/profiles/r1* .snap/profiles/r2* .snap/profiles/r3 .snap/profiles/r4 .snap/BENCH_r* .snap/GPUTEST_r* \
       .snap/MULTICHIP_r* .snap/SCALE_r* .snap/SURVEY.md .snap/PAPERS.md .snap/SNIPPETS.md .snap/profiles/r6/r7* .snap/profiles/r6/r8*
for f in nusiprop_amd/libnusi.so nusiprop_amd/tools/phiphi_text_to_binary oracle/_build/libnusi_oracle.so \
         tests/_build/libhostcheck.so scripts/calib/pmc_calib scripts/dev/gsl_bench; do
  [ -e "$f" ] && { mkdir -p ".snap/$(dirname "$f")"; cp -p "$f" ".snap/$f"; }
done
git rev-parse --short HEAD > .snap/SNAP_HEAD
for f in build/variants/libnusi_*.so; do   # A/B variants (scripts/build_variant.sh), if any
  [ -e "$f" ] && { mkdir -p .snap/build/variants; cp -p "$f" ".snap/$f"; }
done
echo "snap: $(cat .snap/SNAP_HEAD) -> .snap"
