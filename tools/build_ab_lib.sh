#!/bin/bash
# Build the library of a git revision (default HEAD) into ablib/libcwdm_<name>.so for
# same-box A/B runs (CWDM_LIB=... CWDM_ALLOW_STALE_LIB=1).  usage: tools/build_ab_lib.sh NAME [REV [MAKEVARS...]]
# (e.g. tools/build_ab_lib.sh stamps HEAD STAMPS=1: the s_memtime diagnostics build)
set -e
NAME=$1; REV=${2:-HEAD}; shift; shift || true
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/fast-cwdm_amd $T/include
git -C $R archive $REV fast-cwdm_amd/csrc fast-cwdm_amd/cwdm_hip include | tar -x -C $T
make -C $T/fast-cwdm_amd/csrc -j8 "$@" > $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
mkdir -p $R/ablib
cp $T/fast-cwdm_amd/lib/libcwdm.so $R/ablib/libcwdm_$NAME.so
rm -rf $T
echo $R/ablib/libcwdm_$NAME.so
