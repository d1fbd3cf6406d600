"""Build ``libclasfv.so`` (all HIP kernels + the C ABI) for gfx950 with hipcc, in-tree.

The shared library lands next to this file so it travels with the repository snapshot to the GPU
box (a JIT cache under ~/.cache would not). The build embeds a content hash of its sources
(``clasfv_source_hash()``); the library counts as up to date only when that hash equals the hash of
the sources on disk, so a prebuilt binary older than its sources is never used (file times are not
trusted: a snapshot can carry any mtime).
"""
import hashlib
import os
import re
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
INCLUDE = os.path.join(REPO_DIR, "include")
LIB_PATH = os.path.join(PKG_DIR, "libclasfv.so")
SOURCES = ["engine.hip", "conv.hip", "conv_patch.hip", "winograd.hip", "winograd2.hip", "winograd4.hip", "winograd4w.hip",
           "winograd_t.hip", "decoder.hip", "plumbing.hip", "twalk.hip"]
HEADERS = ["common.h", "plumbing.h", "wino4_common.h"]
ARCH = os.environ.get("CLASFV_OFFLOAD_ARCH", "gfx950")
# Per-file extra flags. winograd_t.hip: no SLP vectorisation -- packed f32 VALU (v_pk_*) beside
# MFMAs costs issue cycles and the pack/unpack moves doubled the temporal kernel's vector stream.
EXTRA_FLAGS = {"winograd_t.hip": ["-fno-slp-vectorize"]}


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the CLAS-FV engine needs ROCm's hipcc to build libclasfv.so")


def _inputs():
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files.append(os.path.join(INCLUDE, "clasfv.h"))
    return files


HASH_MARK = b"clasfv-source-hash:"


def source_hash():
    """16 hex digits of SHA-256 over the names and bytes of every build input, the compile flags
    included (what clasfv_source_hash() of a library built from them returns after the mark)."""
    h = hashlib.sha256()
    h.update(repr((ARCH, sorted(EXTRA_FLAGS.items()))).encode())
    for f in _inputs():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def library_hash(path=LIB_PATH):
    """The source hash embedded in a built library (read from its bytes, without loading it), or
    None when the file is missing or carries no hash."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        m = re.search(re.escape(HASH_MARK) + rb"([0-9a-f]{16})", fh.read())
    return m.group(1).decode() if m else None


def up_to_date():
    return library_hash() == source_hash()


def build(force=False, verbose=False):
    """Compile the engine. Returns the library path. Each source is compiled to an object in
    parallel (every kernel is launched from its own translation unit, so no relocatable device
    code is needed), then the objects are linked into one shared library.

    Concurrent callers (e.g. every rank of a torchrun job finding no library) are serialised by an
    exclusive lock on build.lock; each build compiles into its own temporary directory and the
    finished library replaces the old one atomically."""
    if not force and up_to_date():
        return LIB_PATH
    import fcntl
    with open(os.path.join(PKG_DIR, "build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and up_to_date():  # another process built it while this one waited
            return LIB_PATH
        return _build_locked(verbose)


def _build_locked(verbose):
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(os.path.join(PKG_DIR, "build_obj"), exist_ok=True)
    objdir = tempfile.mkdtemp(prefix="build-", dir=os.path.join(PKG_DIR, "build_obj"))
    hipcc = _hipcc()
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", INCLUDE]
    digest = source_hash()

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        extra = list(EXTRA_FLAGS.get(src, []))
        if src == "engine.hip":
            extra.append(f'-DCLASFV_SOURCE_HASH="{digest}"')
        cmd = [hipcc] + flags + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src} ({r.returncode}):\n{r.stderr[-6000:]}")
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    try:
        with ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(compile_one, SOURCES))
        tmp = os.path.join(objdir, "libclasfv.so")
        r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs,
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed ({r.returncode}):\n{r.stderr[-6000:]}")
        os.replace(tmp, LIB_PATH)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
