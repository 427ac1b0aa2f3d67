"""Stamp committed PMC summaries with the per-group kernel-source digests (bench.KERNEL_GROUPS)
of the tree they were collected at, so that bench.py can tell which of their figures still
describe the running kernels (a change to the NMS kernel leaves the CNN counters valid).

    python tools/pmc_stamp.py --commit 97ccab3 profiles/round5/r5e/pmc/report.json ...

--commit: read the kernel sources of that commit (git show); without it, the working tree's (what
tools/pmc_round.sh does on the GPU box).  The file's existing kernel_src_sha must equal that tree's
full digest -- the check that the commit is the one the counters were taken at."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--commit", default=None)
    ap.add_argument("files", nargs="+")
    a = ap.parse_args()
    read = None
    if a.commit:
        def read(name):
            return subprocess.run(["git", "-C", ROOT, "show",
                                   "%s:openpose_amd/csrc/kernels/%s" % (a.commit, name)],
                                  check=True, capture_output=True).stdout
        ls = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", a.commit,
                             "openpose_amd/csrc/kernels/"], check=True, capture_output=True,
                            text=True).stdout.split()
        names = sorted(os.path.basename(p) for p in ls)
        import hashlib
        h = hashlib.sha256()
        for f in names:
            h.update(f.encode() + b"\0" + read(f))
        full = h.hexdigest()[:16]
    else:
        full = bench.kernel_src_sha()
    for path in a.files:
        with open(path) as f:
            d = json.load(f)
        if d.get("kernel_src_sha") not in (None, full):
            sys.exit("%s: kernel_src_sha %s is not the digest of %s (%s)"
                     % (path, d.get("kernel_src_sha"), a.commit or "the working tree", full))
        d["kernel_src_sha"] = full
        for g in bench.KERNEL_GROUPS:
            d["%s_kernel_src_sha" % g] = bench.kernel_src_sha(g, read)
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
        print(path, {k: v for k, v in d.items() if k.endswith("kernel_src_sha")})


if __name__ == "__main__":
    main()
