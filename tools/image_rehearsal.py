#!/usr/bin/env python3
"""Rehearse docker/Dockerfile without a container engine (none is available in CI
containers or here): replay its stages on scratch directories and check the result.

* the build context is the repository minus .dockerignore;
* every stage gets its own root directory; absolute paths of COPY / WORKDIR / ENV are
  mapped under that root;
* RUN commands execute with bash in the stage's WORKDIR. Package installation
  (apt-get / pip) is skipped: it needs the network and only provides the toolchain and
  Python packages this machine already has;
* then the image's entrypoint is run as the DaemonSet runs it (`--help` instead of
  serving), with the install destination redirected, and the installed files checked.

    python tools/image_rehearsal.py [--keep DIR]

Exit status 0 = the image would build and its entrypoint would start.
"""
import argparse
import fnmatch
import os
import shlex
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_PREFIXES = ("apt-get", "pip3 install", "pip install", "rm -rf /var/lib/apt")


def dockerignore(ctx_root):
    path = os.path.join(ctx_root, ".dockerignore")
    if not os.path.exists(path):
        return []
    return [l.strip() for l in open(path) if l.strip() and not l.startswith("#")]


def ignored(rel, patterns):
    for p in patterns:
        p = p.rstrip("/")
        if p.startswith("**/"):
            if any(fnmatch.fnmatch(part, p[3:]) for part in rel.split("/")):
                return True
        elif rel == p or rel.startswith(p + "/") or fnmatch.fnmatch(rel, p) or fnmatch.fnmatch(
                os.path.basename(rel), p):
            return True
    return False


def make_context(dst):
    pats = dockerignore(REPO)
    for dirpath, dirnames, filenames in os.walk(REPO):
        rel_dir = os.path.relpath(dirpath, REPO)
        rel_dir = "" if rel_dir == "." else rel_dir
        dirnames[:] = [d for d in dirnames if not ignored(os.path.join(rel_dir, d) if rel_dir else d, pats)]
        for f in filenames:
            rel = os.path.join(rel_dir, f) if rel_dir else f
            if ignored(rel, pats):
                continue
            os.makedirs(os.path.join(dst, rel_dir), exist_ok=True)
            shutil.copy2(os.path.join(REPO, rel), os.path.join(dst, rel), follow_symlinks=False)


def instructions(dockerfile):
    """(keyword, argument) pairs with line continuations joined and comments dropped."""
    out, cur = [], ""
    for line in open(dockerfile):
        s = line.rstrip("\n")
        if not cur and (not s.strip() or s.lstrip().startswith("#")):
            continue
        if s.endswith("\\"):
            cur += s[:-1] + " "
            continue
        cur += s
        kw, _, arg = cur.strip().partition(" ")
        out.append((kw.upper(), arg.strip()))
        cur = ""
    return out


class Stage:
    def __init__(self, root, name):
        self.root, self.name, self.workdir, self.env = root, name, "/", {}
        os.makedirs(root, exist_ok=True)

    def path(self, p):
        p = p if p.startswith("/") else os.path.join(self.workdir, p)
        return os.path.join(self.root, p.lstrip("/"))


def copy(src, dst, into_dir):
    if os.path.isdir(src):
        shutil.copytree(src, dst, dirs_exist_ok=True, symlinks=True)
    else:
        if into_dir or dst.endswith("/"):
            os.makedirs(dst, exist_ok=True)
            dst = os.path.join(dst, os.path.basename(src))
        else:
            os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy2(src, dst)


def rehearse(work, log=print):
    ctx = os.path.join(work, "context")
    make_context(ctx)
    args, stages, st = {}, {}, None
    for kw, arg in instructions(os.path.join(ctx, "docker", "Dockerfile")):
        if kw == "ARG":
            k, _, v = arg.partition("=")
            args[k] = v
        elif kw == "FROM":
            parts = arg.split()
            name = parts[2] if len(parts) >= 3 and parts[1].upper() == "AS" else f"stage{len(stages)}"
            st = Stage(os.path.join(work, name), name)
            stages[name] = st
            log(f"FROM {parts[0]} -> {st.root}")
        elif kw == "WORKDIR":
            st.workdir = arg
            os.makedirs(st.path(arg), exist_ok=True)
        elif kw == "ENV":
            for tok in shlex.split(arg):
                k, _, v = tok.partition("=")
                st.env[k] = v
        elif kw == "COPY":
            toks = arg.split()
            src_root = ctx
            if toks[0].startswith("--from="):
                src_root = stages[toks[0].split("=", 1)[1]].root
                toks = toks[1:]
            *srcs, dst = toks
            for s in srcs:
                src = os.path.join(src_root, s.lstrip("/"))
                if not os.path.exists(src):
                    raise RuntimeError(f"COPY source missing: {s}")
                copy(src, st.path(dst), into_dir=len(srcs) > 1)
            log(f"COPY {' '.join(srcs)} {dst}")
        elif kw == "RUN":
            for seg in [s.strip() for s in arg.split("&&")]:
                if seg.startswith(SKIP_PREFIXES):
                    log(f"RUN (skipped, package install) {seg[:60]}")
                    continue
                log(f"RUN {seg[:100]}")
                p = subprocess.run(["bash", "-c", seg], cwd=st.path(st.workdir), capture_output=True, text=True,
                                   env=dict(os.environ, **args))
                if p.returncode:
                    raise RuntimeError(f"RUN failed ({p.returncode}): {seg}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}")
        elif kw == "ENTRYPOINT":
            st.entrypoint = shlex.split(arg.strip("[]").replace(",", " ").replace('"', ""))
    return stages, st


def check_runtime(final, work, log=print):
    lib = final.path("/opt/amd-vgpu/4paradigm-k8s-device-plugin_amd/lib")
    for f in ("libvgpu_hip.so", "libvgpu_region.so", "vgpuctl", "vgpu-ledger", "vgpu-validate", "ld.so.preload"):
        if not os.path.exists(os.path.join(lib, f)):
            raise RuntimeError(f"image lacks {f}")
    dest = os.path.join(work, "host-usr-local-vgpu")
    env = dict(os.environ)
    env.update({k: v.replace("/opt/amd-vgpu", final.path("/opt/amd-vgpu")) for k, v in final.env.items()})
    env.update(VGPU_LIB_DIR=lib, VGPU_DIR=dest)
    entry = final.path(final.entrypoint[0])
    p = subprocess.run(["bash", entry, "--help"], env=env, capture_output=True, text=True, timeout=120)
    if p.returncode:
        raise RuntimeError(f"entrypoint failed ({p.returncode}): {p.stderr[-2000:]}")
    for f in ("libvgpu_hip.so", "libvgpu_region.so", "vgpuctl", "ld.so.preload"):
        if not os.path.exists(os.path.join(dest, f)):
            raise RuntimeError(f"entrypoint did not install {f}")
    for d in ("shared", "lock", "allowlist/containers"):
        if not os.path.isdir(os.path.join(dest, d)):
            raise RuntimeError(f"entrypoint did not create {d}/")
    lock = os.path.join(dest, "lock", "hostpid.lock")
    if not os.path.isfile(lock) or os.stat(lock).st_mode & 0o777 != 0o644:
        raise RuntimeError("entrypoint did not create the read-only host-PID lock file (0644)")
    # The installed shim is a loadable ELF exporting the interposed entry points.
    nm = subprocess.run(["nm", "-D", "--defined-only", os.path.join(dest, "libvgpu_hip.so")], capture_output=True,
                        text=True)
    for sym in ("hsa_amd_memory_pool_allocate", "hipLaunchKernel", "amdsmi_get_gpu_memory_total"):
        if sym not in nm.stdout:
            raise RuntimeError(f"installed shim lacks {sym}")
    log(f"entrypoint --help ok; installed into {dest}: {sorted(os.listdir(dest))}")
    return p.stdout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keep", default=None, help="work directory to keep (default: a temporary one)")
    a = ap.parse_args()
    work = a.keep or tempfile.mkdtemp(prefix="image-rehearsal-")
    try:
        stages, final = rehearse(work)
        check_runtime(final, work)
        print("image rehearsal: OK")
    finally:
        if not a.keep:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
