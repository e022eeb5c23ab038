"""Build the native extension in-tree: ``quorum_amd/_qmx<EXT_SUFFIX>``.

Every translation unit is compiled by ``hipcc -x hip --offload-arch=gfx950`` (host code for
the CPU engine, device code for the CDNA4 kernels) and linked into one pybind11 module,
so the built ``.so`` travels with the repo snapshot to the GPU box.

    python -m quorum_amd.ops.build [--debug] [--jobs N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "qmx"
SOURCES = ["qmx_engine.cpp", "qmx_json.cpp", "qmx_server.cpp", "qmx_exchange.cpp", "qmx_prof.cpp", "qmx_hip.hip",
           "bindings.cpp"]
ARCH = os.environ.get("QMX_ARCH", "gfx950")


def _digest(*parts) -> str:
    """Build key: every input that changes the output (source and header bytes, the exact
    command line with its flags and target arch, the compiler binary)."""
    import hashlib

    h = hashlib.sha256()
    for p in parts:
        if isinstance(p, Path):
            h.update(p.read_bytes())
        else:
            h.update(str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def _compiler_id(cc: str) -> str:
    real = os.path.realpath(cc)
    st = os.stat(real)
    return f"{real}:{st.st_size}:{int(st.st_mtime)}"


def _fresh(out: Path, key: str) -> bool:
    k = out.with_name(out.name + ".key")
    return out.exists() and k.exists() and k.read_text() == key


def _stamp(out: Path, key: str) -> None:
    out.with_name(out.name + ".key").write_text(key)


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build quorum_amd)")


def ext_path() -> Path:
    return PKG / ("_qmx" + sysconfig.get_config_var("EXT_SUFFIX"))


def _flags(debug: bool):
    import pybind11

    inc = [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    return inc + opt + ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
                        "-fvisibility=hidden"]


class _BuildLock:
    """Inter-process lock so concurrent ranks never race on the in-tree .so/.o files."""

    def __enter__(self):
        import fcntl

        BUILD.mkdir(parents=True, exist_ok=True)
        self.f = open(BUILD / ".lock", "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        import fcntl

        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def build(debug: bool = False, jobs: int = 3, verbose: bool = False) -> Path:
    with _BuildLock():
        return _build(debug, jobs, verbose)


def _build(debug: bool = False, jobs: int = 3, verbose: bool = False) -> Path:
    cc = hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    flags = _flags(debug)
    out = ext_path()
    headers = sorted(CSRC.glob("*.h"))
    cid = _compiler_id(cc)

    def obj(src: str):
        s = CSRC / src
        o = BUILD / (src + ".o")
        cmd = [cc, "-x", "hip", "-c", str(s), "-o", str(o)] + flags
        key = _digest(cid, " ".join(cmd), s, *headers)  # content + flags + arch, not mtimes
        if _fresh(o, key):
            return o, key
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        _stamp(o, key)
        return o, key

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        built = list(ex.map(obj, SOURCES))
    objs = [o for o, _ in built]
    cmd = [cc, "-shared", "-o", str(out)] + [str(o) for o in objs] + [
        f"--offload-arch={ARCH}", "-fPIC", "-L/opt/rocm/lib", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", "-lssl", "-lcrypto", "-Wl,-rpath,/opt/rocm/lib"]
    key = _digest(cid, " ".join(cmd), *[k for _, k in built])
    if _fresh(out, key):
        return out
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    _stamp(out, key)
    return out


TOOLS = {"qmx_mock": "mock_backend.cpp", "qmx_loadgen": "loadgen.cpp"}
BIN = PKG / "bin"


def build_tools(verbose: bool = False) -> list:
    """Host-only C++ tools (mock backend, load generator) -> quorum_amd/bin/."""
    with _BuildLock():
        return _build_tools(verbose)


def _build_tools(verbose: bool = False) -> list:
    BIN.mkdir(exist_ok=True)
    out = []
    cxx = shutil.which("g++") or shutil.which("c++")
    for name, src in TOOLS.items():
        s = PKG / "tools" / "csrc" / src
        b = BIN / name
        out.append(b)
        cmd = [cxx, "-O2", "-std=c++17", "-pthread", str(s), "-o", str(b)]
        key = _digest(_compiler_id(cxx), " ".join(cmd), s)
        if _fresh(b, key):
            continue
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"tool build failed: {src}\n{r.stderr}")
        _stamp(b, key)
    return out


# Sanitizer builds of the host runtime.  Device code is never sanitized:
# every -fsanitize= goes after -Xarch_host so hipcc applies it to host compilation only.
SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]
SAN_TARGETS = {
    "qmx_fuzz_asan": (["tools/csrc/fuzz_host.cpp", "csrc/qmx_engine.cpp", "csrc/qmx_json.cpp"], []),
    "qmx_server_asan": (["tools/csrc/server_main.cpp", "csrc/qmx_server.cpp", "csrc/qmx_engine.cpp",
                         "csrc/qmx_json.cpp", "csrc/qmx_exchange.cpp", "csrc/qmx_prof.cpp", "csrc/qmx_hip.hip"],
                        ["-L/opt/rocm/lib", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", "-lssl", "-lcrypto",
                         "-Wl,-rpath,/opt/rocm/lib", "-pthread"]),
}


def build_sanitized(verbose: bool = False) -> list:
    """ASan+UBSan host builds -> quorum_amd/bin/qmx_fuzz_asan, qmx_server_asan."""
    with _BuildLock():
        BIN.mkdir(exist_ok=True)
        cc = hipcc()
        headers = sorted(CSRC.glob("*.h"))
        out = []

        def one(item):
            name, (srcs, libs) = item
            b = BIN / name
            paths = [PKG / x for x in srcs]
            cmd = [cc, "-x", "hip", f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", f"-I{CSRC}"] + SAN_FLAGS + \
                [str(x) for x in paths] + ["-o", str(b), "-fsanitize=address", "-fsanitize=undefined"] + libs
            key = _digest(_compiler_id(cc), " ".join(cmd), *paths, *headers)
            if _fresh(b, key):
                return b
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"sanitizer build failed: {name}\n{r.stderr[-4000:]}")
            _stamp(b, key)
            return b

        with cf.ThreadPoolExecutor(max_workers=2) as ex:
            out = list(ex.map(one, SAN_TARGETS.items()))
        return out


# ThreadSanitizer build of the data plane (host code only): io loops, the shared engine's tick
# lanes, verify shadow, metrics — the threads that share slot tables and result queues.
TSAN_FLAGS = ["-Xarch_host", "-fsanitize=thread", "-Xarch_host", "-fno-omit-frame-pointer"]


def build_tsan(verbose: bool = False) -> Path:
    """TSan host build -> quorum_amd/bin/qmx_server_tsan."""
    with _BuildLock():
        BIN.mkdir(exist_ok=True)
        srcs, libs = SAN_TARGETS["qmx_server_asan"]
        b = BIN / "qmx_server_tsan"
        paths = [PKG / x for x in srcs]
        cc = hipcc()
        cmd = [cc, "-x", "hip", f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", f"-I{CSRC}"] + TSAN_FLAGS + \
            [str(x) for x in paths] + ["-o", str(b), "-fsanitize=thread"] + libs
        key = _digest(_compiler_id(cc), " ".join(cmd), *paths, *sorted(CSRC.glob("*.h")))
        if _fresh(b, key):
            return b
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"tsan build failed\n{r.stderr[-4000:]}")
        _stamp(b, key)
        return b


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="also build the ASan/UBSan and TSan host binaries")
    args = ap.parse_args(argv)
    path = build(args.debug, args.jobs, args.verbose)
    print(path)
    for t in build_tools(args.verbose):
        print(t)
    if args.sanitize:
        for t in build_sanitized(args.verbose):
            print(t)
        print(build_tsan(args.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
