#!/bin/bash
# Build libfmpnp.so with extra compiler flags into ab_old/<name>/ (A/B measurement builds):
#   tools/build_ab.sh spec -DFMPNP_SPEC=1
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
out=$ROOT/ab_old/$name
mkdir -p "$out"
cd "$ROOT/featuremetric-pnp_amd"
for f in fmpnp_lm fmpnp_lm_f32 fmpnp_lm_f64 fmpnp_pack fmpnp_points fmpnp_api; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -I../include -Icsrc "$@" -c -o "$out/$f.o" csrc/$f.hip &
done
wait
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -o "$out/libfmpnp.so" "$out"/*.o
rm -f "$out"/*.o
echo "built $out/libfmpnp.so"
