"""Build identity of libfmpnp.so without loading it (no torch import): the LM kernel
specialisation a launch plan names, and a digest of the sources the library is built from.
bench.py accepts a committed rocprofv3 profile only when both match the launch it times;
tools/pmc_summary.py records them on the GPU box (which has the tree but no git history)."""
import os


def kernel_name(info):
    """The demangled name of the LM kernel specialisation a launch plan (last_launch() / plan())
    ran: fmpnp::lm_kernel<T, WPS, TEAM, RATIO, VAR>, as rocprofv3 reports it."""
    t = "double" if info["dtype"] == 1 else "float"
    b = lambda v: "true" if v else "false"  # noqa: E731
    return f"fmpnp::lm_kernel<{t}, {info['build']}, {b(info['team'])}, {b(info['ratio'])}, {info['variant']}>"


# the sources libfmpnp.so is built from (kernel code, ABI, build flags)
SOURCE_FILES = ("featuremetric-pnp_amd/Makefile", "featuremetric-pnp_amd/csrc", "include/fmpnp.h")


def source_digest(root=None, flags=""):
    """sha256 (16 hex digits) over the library's source files, path and content, and the compile
    flags (the Makefile passes its effective FLAGS, so a build with other -D options or another
    ARCH gets another digest): identifies the build a profile was taken with on a box that has no
    git history (gpurun ships the tree)."""
    import hashlib
    root = root or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    files = []
    for rel in SOURCE_FILES:
        p = os.path.join(root, rel)
        if os.path.isdir(p):
            files += sorted(os.path.join(rel, f) for f in os.listdir(p)
                            if f.endswith((".hip", ".h", ".cpp")) and os.path.isfile(os.path.join(p, f)))
        elif os.path.isfile(p):
            files.append(rel)
    h = hashlib.sha256()
    for rel in files:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    if flags:
        h.update(b"flags\0" + " ".join(flags.split()).encode())
    return h.hexdigest()[:16]


def library_file_digest(path=None):
    """The digest compiled into a built libfmpnp.so (its fmpnp_build_info string), read from the
    file without loading it: what the profiling tools record, so a profile names the build it
    was taken with, flags included."""
    import re
    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libfmpnp.so")
    try:
        with open(path, "rb") as f:
            m = re.search(rb"source_digest=([0-9a-z]{7,16})", f.read())
    except OSError:
        return "unknown"
    return m.group(1).decode() if m else "unknown"
