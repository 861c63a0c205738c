#!/bin/bash
# Build the working tree's library with the in-kernel stamps (make STAMPS=1) into
# ablib/libcwdm_stamps.so (for CWDM_LIB=... CWDM_ALLOW_STALE_LIB=1 runs).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/fast-cwdm_amd $T/include
cp -r $R/fast-cwdm_amd/csrc $R/fast-cwdm_amd/cwdm_hip $T/fast-cwdm_amd/
cp $R/include/cwdm.h $T/include/
make -C $T/fast-cwdm_amd/csrc -j8 STAMPS=1 > $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
mkdir -p $R/ablib
cp $T/fast-cwdm_amd/lib/libcwdm.so $R/ablib/libcwdm_stamps.so
rm -rf $T
echo $R/ablib/libcwdm_stamps.so
