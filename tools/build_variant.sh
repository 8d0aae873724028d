#!/bin/bash
# Build an experimental libl7match variant: tools/build_variant.sh NAME "-DFLAG ..."
# -> variants/NAME.so (same sources, extra compiler flags); bench.py / tests
# load it with L7M_LIB=variants/NAME.so.
set -eu
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=${2:-}
B=cilium_amd/csrc/build_$NAME
mkdir -p $B variants
for f in regex_ecma regex_re2 regex_vm dfa_pack http_compile kafka_compile l7m_api l7m_side l7m_batch l7m_multi; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -pthread -Wall -Wno-unused-result $FLAGS -D__HIP_PLATFORM_AMD__ \
    -I/opt/rocm/include -x c++ -c cilium_amd/csrc/$f.cc -o $B/$f.o &
done
for f in l7m_kernels l7m_kafka; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -pthread -Wall -Wno-unused-result $FLAGS --offload-arch=gfx950 \
    -munsafe-fp-atomics -c cilium_amd/csrc/$f.hip -o $B/$f.o &
done
for F in 0 1 2 3; do  # the HTTP feature-set translation units (Makefile FEAT_OBJS)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -pthread -Wall -Wno-unused-result $FLAGS --offload-arch=gfx950 \
    -munsafe-fp-atomics -DL7M_FEAT=$F -c cilium_amd/csrc/l7m_http_feat.hip -o $B/l7m_http_f$F.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o variants/$NAME.so $B/*.o -ldl
echo "built variants/$NAME.so"
