#!/bin/bash
# f-only pack tile sweep (FMPNP_PACK_F_CT x FMPNP_PACK_F_XT) on the BASELINE shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for ct in 64 128; do for xt in 32 64; do
  echo "CT=$ct XT=$xt"; FMPNP_PACK_F_CT=$ct FMPNP_PACK_F_XT=$xt timeout -k 10 120 python3 tools/bench_pack_f.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done
