# Build the committed tree's library (git HEAD) under alt_lib/head/ for A/B runs against the
# working tree (tools/ab_bdf.sh head).
set -euo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/alt_lib/head
rm -rf "$dst"
mkdir -p "$dst"
git -C "$root" archive HEAD include odelib_amd/csrc | tar -x -C "$dst"
make -s -C "$dst/odelib_amd/csrc" -j8 libodelib_amd.so
echo "$dst/odelib_amd/csrc/libodelib_amd.so"
