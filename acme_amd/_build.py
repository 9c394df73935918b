"""Builds libacme_hip.so (gfx950) in-tree with hipcc.

No CMake / torch extension machinery: each .hip translation unit is compiled to an
object with `hipcc --offload-arch=gfx950` (in parallel) and linked into one shared
library next to this file, so it travels to the GPU box with the repository snapshot.
"""

import concurrent.futures
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
# ACME_BUILD_OUT / ACME_BUILD_OBJDIR: an experiment's variant library (e.g. with
# ACME_EXTRA_CFLAGS=-DP3_FOUR_TERMS=1), loaded through ACME_LIB_PATH.
LIB = os.environ.get("ACME_BUILD_OUT") or os.path.join(HERE, "libacme_hip.so")
OBJDIR = os.environ.get("ACME_BUILD_OBJDIR") or os.path.join(HERE, "csrc", "build")
ARCH = os.environ.get("ACME_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
          "-Wall", "-Wno-unused-result"] + os.environ.get("ACME_EXTRA_CFLAGS", "").split()


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return sorted(hs)


def _digest(paths):
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()


def _compile(src, hdr_digest):
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    stamp = obj + ".sha"
    key = _digest([src]) + hdr_digest
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == key:
        return obj
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(key)
    return obj


def build(verbose: bool = True) -> str:
    """Compiles (incrementally) and links libacme_hip.so; returns its path."""
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    hdr = _digest(_headers())
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr), srcs))
    key = _digest(objs)
    stamp = LIB + ".sha"
    if not (os.path.exists(LIB) and os.path.exists(stamp) and open(stamp).read() == key):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        with open(stamp, "w") as f:
            f.write(key)
    if verbose:
        print(f"[acme_amd] built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build()
