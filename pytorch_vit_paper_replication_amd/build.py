"""In-tree native build of the gfx950 extension (``_C``).

The HIP kernels (``csrc/*.hip``) are compiled by ``hipcc --offload-arch=gfx950`` into object files
without any torch headers; only ``csrc/bindings.cpp`` sees ATen/pybind11 and is compiled by the host
C++ compiler. Everything is linked into ``pytorch_vit_paper_replication_amd/_C<EXT_SUFFIX>`` next to
this file so that the built library travels with the source tree (and is what the GPU box loads).

Rebuilds are incremental (per-object source/header mtime check) and the objects compile in parallel.
Run ``python -m pytorch_vit_paper_replication_amd.build`` (or ``build_extension()``) to build.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR / "_build"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
if ARCH != "gfx950":  # this framework is written for CDNA4 only
    ARCH = "gfx950"


def ext_path(debug: bool = False) -> Path:
    return PKG_DIR / (("_C_debug" if debug else "_C") + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_dirs():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    return tdir / "include", tdir / "lib"


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return str(Path(rocm) / "bin" / "hipcc")


HASH_TAG = b"PVR_SRC_HASH="


def source_hash(csrc: Path = CSRC) -> str:
    """Content hash of every native source (``csrc/*.hip|*.h|*.cpp``, by name and bytes): the
    identity compiled into ``_C`` so that :mod:`._ext` can refuse a binary built from other sources."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(p for p in Path(csrc).iterdir() if p.suffix in (".hip", ".h", ".cpp")):
        h.update(f.name.encode() + b"\0")
        h.update(f.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:16]


def embedded_hash(so: Path) -> str | None:
    """The source hash a built ``_C`` carries (read from the file, without importing it)."""
    try:
        data = Path(so).read_bytes()
    except OSError:
        return None
    i = data.find(HASH_TAG)
    if i < 0:
        return None
    return data[i + len(HASH_TAG):i + len(HASH_TAG) + 16].decode("ascii", "replace")


def _newer(src_files, target: Path) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(s).stat().st_mtime > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build command failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_extension(verbose: bool = False, force: bool = False, jobs: int | None = None, debug: bool = False,
                    extra_flags: tuple = ()) -> Path:
    """Compile every HIP kernel for gfx950 and link the torch extension. Returns the .so path.

    ``extra_flags``: additional hipcc flags for experiment builds (CLI: ``--hipcc-flag=-DFOO``); pass
    ``force=True`` with them, since the incremental check compares timestamps only.

    ``debug=True`` builds ``_C_debug`` (separate objects) with ``-DPVR_DEBUG``: device-side
    ``PVR_ASSERT`` invariant checks in the kernels; load it with ``PVR_DEBUG_KERNELS=1``."""
    build_dir = BUILD_DIR.with_name("_build_debug") if debug else BUILD_DIR
    build_dir.mkdir(exist_ok=True)
    ext_name = "_C_debug" if debug else "_C"
    dbg_flags = ["-DPVR_DEBUG"] if debug else []
    inc, lib = _torch_dirs()
    py_inc = sysconfig.get_paths()["include"]
    headers = list(CSRC.glob("*.h"))
    hip_srcs = sorted(CSRC.glob("*.hip"))
    objs = []
    jobs_list = []
    hip_flags = [
        f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
        "-munsafe-fp-atomics", "-Wno-unused-result",
        # a kernel parameter shadowed by a local array faulted a GPU in round 3: shadowing is an error
        "-Wshadow", "-Werror=shadow",
    ] + list(extra_flags)
    for src in hip_srcs:
        obj = build_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _newer([src, *headers], obj):
            jobs_list.append([_hipcc(), *hip_flags, *dbg_flags, "-c", str(src), "-o", str(obj)])
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cxx = os.environ.get("CXX", "g++")
    for cpp in sorted(CSRC.glob("*.cpp")):  # host-only translation units (ATen / pybind11 / RCCL)
        obj = build_dir / (cpp.stem + ".o")
        objs.append(obj)
        if force or _newer([cpp, *headers], obj):
            jobs_list.append([
                cxx, "-O2", "-std=c++17", "-fPIC", "-c", str(cpp), "-o", str(obj),
                "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                f"-DTORCH_EXTENSION_NAME={ext_name}", "-DTORCH_API_INCLUDE_EXTENSION_H", *dbg_flags,
                f"-I{inc}", f"-I{inc / 'torch' / 'csrc' / 'api' / 'include'}", "-I/opt/rocm/include", f"-I{py_inc}",
                "-w",
            ])
    if jobs_list:
        n = jobs or min(len(jobs_list), max(1, (os.cpu_count() or 4)), 16)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for out in ex.map(_run, jobs_list):
                if verbose and out.strip():
                    print(out)
    # the source identity: a tiny C unit holding the tag, regenerated whenever the hash changes
    # (a rebuild from the same sources keeps it, so the incremental check stays exact)
    shash = source_hash()
    hsrc = build_dir / "src_hash.c"
    htext = (f'__attribute__((used)) const char pvr_src_hash_tag[] = "{HASH_TAG.decode()}{shash}";\n'
             'const char* pvr_src_hash(void) { return pvr_src_hash_tag + ' + str(len(HASH_TAG)) + '; }\n')
    if not hsrc.exists() or hsrc.read_text() != htext:
        hsrc.write_text(htext)
    hobj = build_dir / "src_hash.o"
    hash_changed = force or _newer([hsrc], hobj)
    if hash_changed:
        _run([os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-c", str(hsrc), "-o", str(hobj)])
    objs.append(hobj)
    so = ext_path(debug)
    if force or jobs_list or hash_changed or not so.exists() or embedded_hash(so) != shash:
        link = [
            _hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(so),
            f"-L{lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
            f"-Wl,-rpath,{lib}", "-ldl",
        ]
        _run(link)
        if verbose:
            print(f"[build] linked {so}")
    return so


if __name__ == "__main__":
    force = "--force" in sys.argv
    extra = tuple(a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--hipcc-flag="))
    p = build_extension(verbose=True, force=force or bool(extra), debug="--debug" in sys.argv, extra_flags=extra)
    print(p)
