"""Build libzenflow_amd.so in-tree with hipcc for gfx950 (MI355X).

``python -m zenflow_amd.build`` (or ``__graft_entry__.build()``).  The output
lands next to this file so the built library travels with the repository
snapshot to the GPU box.
"""

from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
INCLUDE = HERE.parent / "include"
LIB = HERE / "libzenflow_amd.so"
ARCH = os.environ.get("ZF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["zf_runtime.hip", "zf_rqs.hip", "zf_flow.hip", "zf_flow_x3.hip", "zf_flow_x3_k8.hip", "zf_flow_x3_k16.hip", "zf_flow_x3_k32.hip", "zf_flow_x3_k64.hip", "zf_flow_x3_k64_act.hip", "zf_flow_x3_k8_act.hip", "zf_flow_x3_k16_act.hip", "zf_flow_x3_k32_act.hip", "zf_flow_x3_k8_act2.hip", "zf_flow_x3_k16_act2.hip", "zf_flow_x3_k32_act2.hip", "zf_stats.hip", "zf_rccl.hip", "zf_train.hip", "zf_layered.hip"]
HEADERS = sorted(p.name for p in CSRC.glob("*.h"))

FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    "-Wno-unused-result",
    "-I/opt/rocm/include",
    f"-I{INCLUDE}",
]

# Split-MFMA kernel translation units: no SLP packing of scalar f32 ops into
# v_pk_* (packed f32 VALU beside MFMAs costs more issue than two scalar ops;
# cfg2 -1% kernel time)
X3_FLAGS = ["-fno-slp-vectorize"]


def _src_flags(src: str):
    return X3_FLAGS if src.startswith("zf_flow_x3_k") else []


def _fingerprint() -> str:
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        h.update((CSRC / f).read_bytes())
    h.update((INCLUDE / "zenflow_amd.h").read_bytes())
    h.update(" ".join(FLAGS + X3_FLAGS).encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = True, out: Path = LIB, extra=()) -> Path:
    """Compile every HIP source into one shared library (skip if up to date).
    ``out``/``extra``: tuning builds (e.g. ``-DZF_X3_TRACE=1``) into another file."""
    stamp = out.parent / f".{out.stem}.sha256"
    fp = _fingerprint() + " ".join(extra)
    if not force and out.exists() and stamp.exists() and stamp.read_text() == fp:
        return out
    tmp = out.with_suffix(".so.tmp")
    objdir = HERE.parent / "build" / ("obj" if not extra else "obj_" + hashlib.sha1(" ".join(extra).encode()).hexdigest()[:8])
    objdir.mkdir(parents=True, exist_ok=True)
    compile_flags = [f for f in FLAGS if f != "-shared"] + list(extra)

    hdr = hashlib.sha256(b"".join((CSRC / f).read_bytes() for f in HEADERS) + (INCLUDE / "zenflow_amd.h").read_bytes())

    def _compile(src: str) -> Path:
        obj = objdir / (Path(src).stem + ".o")
        cmd = [HIPCC, *compile_flags, *_src_flags(src), "-c", "-o", str(obj), str(CSRC / src)]
        # per-object stamp (source, every header, the command): unchanged units are not rebuilt
        key = hashlib.sha256(hdr.digest() + (CSRC / src).read_bytes() + " ".join(cmd).encode()).hexdigest()
        ostamp = obj.with_suffix(".o.sha256")
        if not force and obj.exists() and ostamp.exists() and ostamp.read_text() == key:
            return obj
        if verbose:
            print("[zenflow_amd.build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        ostamp.write_text(key)
        return obj

    # one hipcc per translation unit, in parallel (the kernels dominate build time)
    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as pool:
        objs = list(pool.map(_compile, SOURCES))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs), "-ldl"]
    if verbose:
        print("[zenflow_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    stamp.write_text(fp)
    return out


if __name__ == "__main__":
    # python -m zenflow_amd.build [--force] [--out PATH] [-DMACRO=V ...]
    argv = sys.argv[1:]
    o = LIB
    if "--out" in argv:
        i = argv.index("--out")
        o = Path(argv[i + 1]).resolve()
        del argv[i : i + 2]
    build(force="--force" in argv, out=o, extra=[a for a in argv if a.startswith("-D")])
