#!/usr/bin/env python3
"""ISA census of one LM kernel variant by phase (verdict r05 item 1).

Compiles ONE instantiation of lm_kernel (default: the headline, float / latency build / no team /
no ratio / VAR_GM_SPEC_512) to gfx950 assembly with -DFMPNP_ISA_MARKS=1, which turns every tl_stamp site of
fmpnp_lm_impl.h into an assembly comment ';@@TL k', then counts the instructions between consecutive
markers (in layout order) by class.  Straight-line phases (projection, loss, partials, combine,
solve) are counted exactly; loops (the gathers) are counted once per static copy.

usage: tools/isa_census.py [--var VAR_GM_SPEC_512] [--ratio 0|1] [--extra '-DFOO=1'] [--out FILE] [--asm FILE]
                           [--rev GIT_REV]   (--rev: the sources of that revision, e.g. round 5's final)
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "featuremetric-pnp_amd")

# tl_stamp sites (fmpnp_lm_impl.h) -> phase names
SITES = {
    0: "evaluation start (pose read)", 1: "projection + memo check done", 2: "gathers done",
    3: "loss + block partial done", 4: "before barrier 1", 5: "after barrier 1",
    6: "combine done", 12: "stepper operands read", 13: "step solved", 14: "decision",
    7: "books kept (team tail)", 8: "pose update start", 9: "tail done", 10: "speculation done",
    11: "after barrier 2", 15: "ratio check done",
}


def classify(op, args, spill_vgprs=frozenset()):
    if op.startswith(("v_fma_f64", "v_fmac_f64", "v_mul_f64", "v_add_f64", "v_max_f64", "v_min_f64",
                      "v_rcp_f64", "v_div_", "v_ldexp_f64", "v_frexp", "v_rndne_f64", "v_fract_f64",
                      "v_trunc_f64", "v_floor_f64", "v_sqrt_f64", "v_rsq_f64", "v_mul_f32", "v_fma_f32",
                      "v_fmac_f32", "v_add_f32", "v_sub_f32", "v_max_f32", "v_min_f32", "v_rcp_f32",
                      "v_floor_f32", "v_fract_f32", "v_rndne_f32", "v_subrev_f32", "v_pk_")):
        return "fp arithmetic"
    if op.startswith("v_cvt"):
        return "conversion"
    if op.startswith("v_readlane") or op.startswith("v_writelane"):
        # to / from an SGPR: the SGPR spill slots live in VGPR lanes (v_writelane = spill, v_readlane from a
        # spill VGPR = reload); other v_readlane are lane reads (the tail's rlane(), the LU fallback's rows)
        vs = [a.strip() for a in args.split(",")]
        if op.startswith("v_writelane") or (len(vs) > 1 and vs[1] in spill_vgprs):
            return "sgpr spill/reload (v_readlane/v_writelane)"
        return "cross-lane (dpp/permlane/readfirstlane)"
    if "_dpp" in op or op.startswith(("v_permlane", "ds_swizzle", "ds_bpermute", "v_readfirstlane")):
        return "cross-lane (dpp/permlane/readfirstlane)"
    if op.startswith(("v_mov", "v_cndmask")):
        return "vector move / select"
    if op.startswith("v_cmp") or op.startswith("v_cmpx"):
        return "vector compare"
    if op.startswith(("global_", "flat_", "buffer_", "scratch_")):
        return "vector memory"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("v_"):
        return "vector integer / address / other"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_setprio")):
        return "wait / nop / barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if "exec" in args:
        return "exec mask (SALU)"
    if op.startswith("s_"):
        return "SALU other"
    return "other"


def compile_asm(var, ratio, extra, out_s, pkg=PKG):
    src = tempfile.NamedTemporaryFile("w", suffix=".hip", delete=False)
    src.write('#include "fmpnp_lm_impl.h"\nnamespace fmpnp {\n'
              f"template __global__ void lm_kernel<float, WPS_LATENCY, false, {'true' if ratio else 'false'}, "
              f"{var}>(LaunchArgs);\n}}\n")
    src.close()
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-I../include", "-Icsrc",
           "-DFMPNP_ISA_MARKS=1", "--cuda-device-only", "-S", src.name, "-o", out_s] + extra.split()
    subprocess.run(cmd, cwd=pkg, check=True, stderr=subprocess.DEVNULL)
    os.unlink(src.name)


def census(asm_path):
    lines = open(asm_path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN5fmpnp9lm_kernel.*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    meta = {}
    for l in lines[end:]:
        m = re.match(r"\s+\.(vgpr_count|sgpr_count|sgpr_spill_count|vgpr_spill_count|agpr_count):\s+(\d+)", l)
        if m:
            meta[m.group(1)] = int(m.group(2))
    spill = frozenset(m.group(1) for l in lines[start:end]
                      for m in [re.match(r"\s+v_writelane_b32 (v\d+),", l)] if m)
    segs = [("kernel entry", collections.Counter())]
    for l in lines[start:end]:
        s = l.strip()
        m = re.match(r";@@TL (\d+)", s)
        if m:
            k = int(m.group(1))
            segs.append((f"TL{k} {SITES.get(k, '')}", collections.Counter()))
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        parts = s.split(None, 1)
        segs[-1][1][classify(parts[0], parts[1] if len(parts) > 1 else "", spill)] += 1
    return meta, segs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", default="VAR_GM_SPEC_512")
    ap.add_argument("--ratio", type=int, default=0)
    ap.add_argument("--extra", default="")
    ap.add_argument("--asm", default=None, help="census an existing .s instead of compiling")
    ap.add_argument("--out", default=None)
    ap.add_argument("--rev", default=None, help="census the sources of this git revision")
    a = ap.parse_args()
    s_path = a.asm or os.path.join(tempfile.gettempdir(), "fmpnp_isa_census.s")
    if not a.asm:
        pkg = PKG
        if a.rev:  # that revision's csrc/ and include/ in a scratch tree
            tmp = tempfile.mkdtemp()
            arch = subprocess.run(["git", "-C", ROOT, "archive", a.rev, "featuremetric-pnp_amd/csrc", "include"],
                                  check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
            pkg = os.path.join(tmp, "featuremetric-pnp_amd")
        compile_asm(a.var, a.ratio, a.extra, s_path, pkg)
    meta, segs = census(s_path)
    classes = sorted({c for _, cnt in segs for c in cnt})
    out = [f"# ISA census: lm_kernel<float, WPS_LATENCY, false, {bool(a.ratio)}, {a.var}> {a.extra}".rstrip()
           + (f" (sources of {a.rev})" if a.rev else ""),
           f"# resources: {meta}",
           "# segments in layout order, each named by the marker that opens it (the code after that tl_stamp "
           "site up to the next marker)"]
    tot = collections.Counter()
    for name, cnt in segs:
        n = sum(cnt.values())
        tot.update(cnt)
        if not n:
            continue
        out.append(f"\n## {name}: {n} instructions")
        for c in classes:
            if cnt[c]:
                out.append(f"   {cnt[c]:5d}  {c}")
    out.append(f"\n## whole kernel (static): {sum(tot.values())} instructions")
    for c in classes:
        out.append(f"   {tot[c]:5d}  {c}")
    text = "\n".join(out) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
