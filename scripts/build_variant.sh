#!/bin/bash
# Build an A/B variant of librfa.so with extra compile flags into abv/librfa_NAME.so
# (own object dir; the in-tree librfa.so is untouched).  Load it with RFA_LIB=abv/librfa_NAME.so.
# Variants are built with -DRFA_AB_BUILD: only they read the RFA_* ablation / stamp variables.
# usage: scripts/build_variant.sh NAME "-DFOO=1 -DBAR=2"
set -eu
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=${2:-}
BASE="-DRFA_AB_BUILD -O3 -fPIC -std=c++20 --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result -fvisibility=hidden"
make -s -C rfanalyzer_amd/csrc -j8 OBJ="$PWD/abv/obj_$NAME" OUT="$PWD/abv/librfa_$NAME.so" HIPFLAGS="$BASE $EXTRA"
ls -la "abv/librfa_$NAME.so"
