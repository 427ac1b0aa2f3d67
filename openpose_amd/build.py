"""Build libopk_hip.so in-tree: every .hip/.cpp under openpose_amd/csrc compiled for gfx950.

    python -m openpose_amd.build [--jobs N]

Objects go to openpose_amd/build/ (git-ignored); the shared library lands at
openpose_amd/libopk_hip.so so it travels with the repo snapshot to the GPU box.
"""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libopk_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

# -ffp-contract=off: the post-processing kernels and the host tables must round every mul/add
# separately to match the CPU path bit for bit; MFMA code is unaffected.
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(HERE, "..", "include")]
DEVICE = ["--offload-arch=" + ARCH, "-munsafe-fp-atomics"]


def sources():
    out = []
    for root, _, files in os.walk(CSRC):
        for f in sorted(files):
            if f.endswith((".hip", ".cpp")):
                out.append(os.path.join(root, f))
    return sorted(out)


def _obj(src, out=OUT):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(out, rel + ".o")


def _compile(src, extra, out=OUT):
    obj = _obj(src, out)
    deps = [src] + [os.path.join(r, f) for r, _, fs in os.walk(CSRC) for f in fs if f.endswith(".h")]
    deps.append(os.path.join(HERE, "..", "include", "opk.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj, None
    cmd = [HIPCC] + COMMON + extra
    if src.endswith(".hip"):
        cmd += ["-x", "hip"] + DEVICE
    cmd += ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, "FAILED %s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr)
    return obj, None


def build(jobs=None, extra=None, verbose=False, out=OUT, lib=LIB):
    """extra/out/lib: dev variant builds (e.g. -D switches into openpose_amd/variants/, loaded
    with OPK_LIB_PATH for A/B runs); the product build uses the defaults."""
    os.makedirs(out, exist_ok=True)
    srcs = sources()
    extra = extra or []
    jobs = jobs or min(8, os.cpu_count() or 1)
    objs, errs = [], []
    with cf.ThreadPoolExecutor(jobs) as ex:
        for obj, err in ex.map(lambda s: _compile(s, extra, out), srcs):
            objs.append(obj)
            if err:
                errs.append(err)
    if errs:
        raise RuntimeError("\n".join(errs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(lib) or os.path.getmtime(lib) < newest:
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", lib] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
        if verbose:
            print("linked", lib)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--variant", default=None, help="dev: name of a variant build in variants/")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="dev: -D for a variant")
    a = ap.parse_args()
    try:
        if a.variant:
            vdir = os.path.join(HERE, "variants")
            print(build(a.jobs, ["-D" + d for d in a.defines], True, os.path.join(vdir, "obj_" + a.variant),
                        os.path.join(vdir, "libopk_%s.so" % a.variant)))
        else:
            print(build(a.jobs, verbose=True))
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
