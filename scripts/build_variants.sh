#!/bin/bash
# Build variants of libska_sdp_hip.so that differ only in wstack.hip compile
# definitions, into exp/<name>.so (git-ignored; loaded via SDP_HIP_LIB_OVERRIDE).
# usage: scripts/build_variants.sh name "-DFOO=1 -DBAR" [name2 "defs2" ...]
set -e
cd "$(dirname "$0")/../ska-sdp-func-python_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../../exp build/var
objs=$(ls build/*.o | grep -v wstack.o)
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=true -I../../include -I. $defs -c wstack.hip -o build/var/$name.o &
done
wait
for o in build/var/*.o; do
  n=$(basename $o .o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/$n.so $objs $o -L/opt/rocm/lib -lhipfft -Wl,-rpath,/opt/rocm/lib
done
rm -rf build/var
ls -la ../../exp
