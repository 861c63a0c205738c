#!/bin/bash
# Host-sanitized build of libcwdm's sources + the plan driver (tests/asan/plan_asan.cpp):
# AddressSanitizer + UBSan on the host side only (-Xarch_host; GPU sanitizers are not
# available on this pool), device code compiled as usual.  Output: $1/plan_asan.
set -e -o pipefail
OUT=$1
R=$(cd "$(dirname "$0")/../.." && pwd)
CS=$R/fast-cwdm_amd/csrc
mkdir -p $OUT
SRCS=$(sed -n '/^SRCS/,/unet_plan.cpp/p' $CS/Makefile | tr -d '\\' | sed 's/SRCS :=//')
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
for f in $SRCS; do echo $f; done | xargs -P ${ASAN_JOBS:-8} -I{} /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g \
  -std=c++17 -fPIC -Wno-unused-command-line-argument $SAN -DCWDM_SRC_HASH=\"asan\" -I$R/include -x hip -c $CS/{} -o $OUT/{}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 $SAN -I$R/include -x hip -c $R/tests/asan/plan_asan.cpp \
  -o $OUT/driver.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $SAN $OUT/*.o -o $OUT/plan_asan
