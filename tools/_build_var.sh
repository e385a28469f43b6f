# Build an experiment variant of the library: tools/_build_var.sh NAME "-DFOO=1 -DBAR=0"
# -> coeb-slam_amd/lib/var_NAME.so (loaded with COEB_LIB_PATH; never a fallback).
set -eu
cd "$(dirname "$0")/../coeb-slam_amd/csrc"
name=$1; defs=${2:-}
out=build/var_$name; mkdir -p $out
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function"
objs=""
for s in $(sed -n "s/^SRCS = //p" Makefile | sed "s/\.hip//g"); do
  /opt/rocm/bin/hipcc $FLAGS $defs -c $s.hip -o $out/$s.o &
  objs="$objs $out/$s.o"
done
wait
make -s build/coeb_tum.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/.tmp_var_$name.so $objs build/coeb_tum.o && mv ../lib/.tmp_var_$name.so ../lib/var_$name.so
echo "built lib/var_$name.so ($defs)"
