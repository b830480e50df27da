#!/bin/bash
# A/B variant of libglsamd.so: the brick-kernel sources (gls_op.hip,
# sweeps.hip) rebuilt with extra flags, linked with the product build's other
# objects into dealii-ns-gls_amd/lib/var/NAME.so (GLS_AMD_LIB selects it;
# .gpurunignore keeps lib/var out of the box push unless a run needs it).
#   bash scripts/build_variant.sh NAME "-DGLS_XDPP_F32=0 ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1
FLAGS=$2
P=dealii-ns-gls_amd
OBJ=/tmp/glsvar_$NAME
mkdir -p $OBJ $P/lib/var
make -s amd
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-parameter -Wno-unused-function"
for f in gls_op sweeps; do
  /opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c -o $OBJ/$f.o $P/csrc/$f.hip &
done
wait
others=$(ls $P/build/*.o | grep -v -e '/gls_op.hip.o' -e '/sweeps.hip.o')
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o $P/lib/var/$NAME.so $OBJ/gls_op.o $OBJ/sweeps.o $others \
  -L/opt/rocm/lib -lrocsolver -lrocblas -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "built $P/lib/var/$NAME.so"
