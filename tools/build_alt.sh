# Build a measurement variant of the library under alt_lib/<name>/ (same sources, extra
# compiler defines), for A/B runs with tools/ab_bench.py (ODELIB_AMD_LIB=...).
#   bash tools/build_alt.sh lds160 -DOE_PIPE_LDS_BYTES=163840
# alt_lib/ is git-ignored; drop ./alt_lib from .gpurunignore while such a run is pending.
set -euo pipefail
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/alt_lib/$name
mkdir -p "$dst/odelib_amd/csrc" "$dst/include"
cp "$root"/include/*.h "$dst/include/"
cp "$root"/odelib_amd/csrc/*.hip "$root"/odelib_amd/csrc/*.cuh "$root"/odelib_amd/csrc/*.h \
   "$root"/odelib_amd/csrc/*.py "$root"/odelib_amd/csrc/Makefile "$dst/odelib_amd/csrc/"
make -s -C "$dst/odelib_amd/csrc" -j8 libodelib_amd.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall $*"
echo "$dst/odelib_amd/csrc/libodelib_amd.so"
