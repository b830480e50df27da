#!/bin/bash
# diagnostic variant libraries of libglsamd.so (timing experiments, CPU side)
# into dealii-ns-gls_amd/lib/var/<name>.so: each line "<name> <-D flags>"
set -eu
cd "$(dirname "$0")/.."
mkdir -p dealii-ns-gls_amd/lib/var
rm -f dealii-ns-gls_amd/lib/var/*.so
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-parameter -Wno-unused-function"
SRC="$(ls dealii-ns-gls_amd/csrc/*.hip dealii-ns-gls_amd/csrc/*.cc)"
LIBS="-L/opt/rocm/lib -lrocsolver -lrocblas -lrccl -Wl,-rpath,/opt/rocm/lib"
while read -r name flags; do
  [ -z "$name" ] && continue
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -shared -o dealii-ns-gls_amd/lib/var/$name.so $SRC $LIBS &
done
wait
ls dealii-ns-gls_amd/lib/var
