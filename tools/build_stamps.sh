#!/bin/bash
# Diagnostic library with in-kernel stamps (never the product library): every
# csrc/*.hip with -DEXO_STAMPS, in parallel, into exo_amd/_lib/libexo_amd_stamps.so
set -e
cd "$(dirname "$0")/../a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd/csrc"
OUT=../exo_amd/_lib
mkdir -p $OUT/stamps
for f in $(grep "^SRCS" Makefile | sed 's/SRCS := //'); do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../../include -I. -DEXO_STAMPS -c -o $OUT/stamps/${f%.hip}.o $f &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libexo_amd_stamps.so $OUT/stamps/*.o
