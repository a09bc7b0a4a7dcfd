"""Build an A/B or diagnostic library from a patched COPY of csrc/ (CPU; the shipped sources stay
untouched, so experiment arms never enter the shipped headers):

    python tools/patch_variant.py OUT.so SPEC.py ENV [ENV ...]          (base: the committed sources, git HEAD)
    MRP_VARIANT_WORKTREE=1 python tools/patch_variant.py ...           (base: the working tree)

SPEC.py defines EDITS = [(file, old, new), ...] (exact text replacements, each `old` must occur
in the file), optionally FLAGS = {"mrp_envE.hip": [...]} (that unit's compile flags instead of
build.py's UNIT_FLAGS entry) and DEFINES = ["NAME", ...] (-D for every unit, e.g. MRP_STAMPS).  Only the listed env units are compiled from the patched copy; the other
units are the default library's objects (python -m gym_puzzles_amd.build first).  Every edit must keep
the LaneState / EnvOps layout (mrp_create checks each unit's compiled dims).
"""
from __future__ import annotations

import os
import runpy
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gym_puzzles_amd import build as B  # noqa: E402


def main():
    out, spec, envs = os.path.abspath(sys.argv[1]), sys.argv[2], [int(e) for e in sys.argv[3:]]
    s = runpy.run_path(spec)
    tag = os.path.splitext(os.path.basename(out))[0]
    work = os.path.join("/tmp", f"mrp_variant_{tag}")
    if os.path.exists(work):
        shutil.rmtree(work)
    if os.environ.get("MRP_VARIANT_WORKTREE"):
        shutil.copytree(os.path.join(ROOT, "gym_puzzles_amd"), os.path.join(work, "gym_puzzles_amd"),
                        ignore=shutil.ignore_patterns("build", "var", "*.so", "__pycache__"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(work, "include"))
    else:   # the committed sources: an A/B against the default library built from HEAD
        os.makedirs(work)
        tar = subprocess.run(["git", "-C", ROOT, "archive", "HEAD", "gym_puzzles_amd", "include"], check=True,
                             capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", work], input=tar, check=True)
    csrc = os.path.join(work, "gym_puzzles_amd", "csrc")
    for f, old, new in s["EDITS"]:
        p = os.path.join(csrc, f)
        txt = open(p).read()
        n = txt.count(old)
        if n == 0:
            raise SystemExit(f"{spec}: edit not found in {f}: {old[:80]!r}")
        open(p, "w").write(txt.replace(old, new))
    B.CSRC = csrc
    B.SOURCES = [os.path.join(csrc, os.path.basename(x)) for x in B.SOURCES]
    B.DEPS = B.SOURCES + [os.path.join(csrc, os.path.basename(x)) for x in B.DEPS if x.endswith(".h")]
    B.UNIT_FLAGS = dict(B.UNIT_FLAGS, **s.get("FLAGS", {}))
    os.environ["MRP_ALLOW_STALE_UNITS"] = "1"
    print(B.build(verbose=True, out=out, only_envs=envs, defines=tuple(s.get("DEFINES", ()))))


if __name__ == "__main__":
    main()
