#!/bin/bash
# Build libfmpnp.so into ab_old/<name>/ for A/B measurements (FMPNP_LIB_PATH selects it):
#   tools/build_ab.sh NAME [REV] [-- extra hipcc flags]
# REV: a git revision whose csrc/ and include/ are built (default: the working tree).
set -e
name=$1; shift
rev=""
if [ $# -gt 0 ] && [ "$1" != "--" ]; then rev=$1; shift; fi
[ "$1" = "--" ] && shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
out=$ROOT/ab_old/$name
mkdir -p "$out"
src=$ROOT/featuremetric-pnp_amd/csrc
inc=$ROOT/include
if [ -n "$rev" ]; then
  tmp=$(mktemp -d)
  mkdir -p "$tmp/csrc" "$tmp/include"
  git -C "$ROOT" archive "$rev" featuremetric-pnp_amd/csrc include | tar -x -C "$tmp"
  src=$tmp/featuremetric-pnp_amd/csrc
  inc=$tmp/include
fi
rm -f "$out"/*.o "$out/libfmpnp.so"
pids=""
for f in fmpnp_lm fmpnp_lm_f32 fmpnp_lm_f64 fmpnp_pack fmpnp_points fmpnp_query fmpnp_api; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -I"$inc" -I"$src" "$@" -c -o "$out/$f.o" "$src/$f.hip" &
  pids="$pids $!"
done
for p in $pids; do wait "$p" || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -o "$out/libfmpnp.so" "$out"/*.o
rm -f "$out"/*.o
echo "built $out/libfmpnp.so ${rev:+from $rev}"
