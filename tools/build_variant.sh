#!/bin/bash
# Link libhkcsa_<name>.so with one source file replaced (A/B on one GPU box: HKCSA_LIB=...):
#   tools/build_variant.sh <name> <file.hip> <replacement path>
set -e
name=$1; file=$2; repl=$3
cd "$(dirname "$0")/../high-order-entropy-compressed-suffix-array_amd/csrc"
obj=../hkcsa/_lib/obj
mkdir -p ../hkcsa/_lib/var
cp "$repl" ../hkcsa/_lib/var/$file
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I/opt/rocm/include -I. -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $FLAGS -c ../hkcsa/_lib/var/$file -o ../hkcsa/_lib/var/${file%.hip}.o
objs=""
for f in hk_sort hk_sa hk_seground hk_bucket hk_bsort hk_wt hk_golomb hk_sample hk_entropy hk_shard hkcsa_abi; do
  if [ "$f.hip" = "$file" ]; then objs="$objs ../hkcsa/_lib/var/$f.o"; else objs="$objs $obj/$f.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 $objs -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o ../hkcsa/_lib/libhkcsa_$name.so
echo "built hkcsa/_lib/libhkcsa_$name.so"
