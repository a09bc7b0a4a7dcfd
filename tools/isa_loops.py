"""Instruction mix of the loops of one kernel in a gfx950 assembly listing (CPU only).

    hipcc <build.py FLAGS> --cuda-device-only -S gym_puzzles_amd/csrc/mrp_env<E>.hip -o env<E>.s
    python tools/isa_loops.py env<E>.s 'k_stepILi<E>ELb0E' [--all]

LLVM annotates every basic block of a loop with its header (`; =>This Inner Loop Header: Depth=d`,
`;   in Loop: Header=BBx_y Depth=d`).  For each loop the blocks that belong to it directly (not to a
loop nested inside it) are summed: instructions, VALU (of which packed v_pk_*, v_readlane,
v_writelane), SALU, s_nop wait states, LDS, branches.  The sweep loops of the solver are the
innermost loops with the most packed VALU; a sweep of NC contact updates issues about
instructions x 4 cycles on a lone wave (MI355X_MICROARCH.md, row 'vector-instruction ISSUE cost'),
so these counts are the issue floor of a sweep as compiled inside k_step.
"""
from __future__ import annotations

import json
import re
import sys
from collections import defaultdict

HDR = re.compile(r"Loop Header: Depth=(\d+)")
MEM = re.compile(r"in Loop: Header=(BB\d+_\d+) Depth=(\d+)")
LBL = re.compile(r"^\.L(BB\d+_\d+):")
BBC = re.compile(r"^; %bb\.(\d+):")


def kernel_lines(path: str, name: str):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        head = ln.split(";")[0].strip()
        if head.endswith(":") and not ln.startswith((".", ";", " ", "\t")) and name in head:
            start = i
            break
    if start is None:
        raise SystemExit(f"no function matching {name!r}")
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def classify(op: str) -> str:
    if op.startswith("v_pk_"):
        return "valu_packed"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane"):
        return "readlane"
    if op.startswith("v_writelane"):
        return "writelane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def analyse(lines):
    blocks = []            # (label, header-of-loop-or-None, depth, is_header, counts)
    cur = {"label": "entry", "loop": None, "depth": 0, "header": False, "n": defaultdict(int), "nop_states": 0}
    for ln in lines:
        s = ln.strip()
        m = LBL.match(ln)
        if m or BBC.match(s):
            blocks.append(cur)
            label = m.group(1) if m else "bb" + BBC.match(s).group(1)
            cur = {"label": label, "loop": None, "depth": 0, "header": False, "n": defaultdict(int), "nop_states": 0}
            h = HDR.search(ln)
            mm = MEM.search(ln)
            if h:
                cur.update(loop=label, depth=int(h.group(1)), header=True)
            elif mm:
                cur.update(loop=mm.group(1), depth=int(mm.group(2)))
            continue
        if s.startswith(";"):
            # continuation lines of a block label's annotation (nested loop headers print their
            # "=> This Inner Loop Header: Depth=d" on a comment line below the label)
            h = HDR.search(s)
            if h and cur["loop"] is None or (h and cur["n"] == {} and not cur["header"]):
                cur.update(loop=cur["label"], depth=int(h.group(1)), header=True)
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        k = classify(op)
        cur["n"][k] += 1
        if k == "s_nop":
            try:
                cur["nop_states"] += int(s.split()[1], 0) + 1
            except (IndexError, ValueError):
                cur["nop_states"] += 1
    blocks.append(cur)
    loops = defaultdict(lambda: {"blocks": 0, "n": defaultdict(int), "nop_states": 0, "depth": 0})
    parent = {}
    for b in blocks:
        if b["loop"] is None:
            continue
        L = loops[b["loop"]]
        L["blocks"] += 1
        L["depth"] = max(L["depth"], b["depth"])
        for k, v in b["n"].items():
            L["n"][k] += v
        L["nop_states"] += b["nop_states"]
    # a loop is innermost if no other loop has a greater depth with blocks between its blocks: use the
    # header annotations: a header at depth d inside loop X appears as `in Loop: Header=X` on its own
    # outer block, which LLVM does not emit, so nesting is read from the header comments' order
    out = []
    for name, L in loops.items():
        n = dict(L["n"])
        instr = sum(n.values())
        out.append({"loop": name, "depth": L["depth"], "blocks": L["blocks"], "instructions": instr,
                    "issue_cycles_lone_wave": 4 * (instr - n.get("s_nop", 0)) + 4 * L["nop_states"],
                    "mix": n, "s_nop_wait_states": L["nop_states"]})
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    res = analyse(kernel_lines(path, name))
    res.sort(key=lambda r: -r["mix"].get("valu_packed", 0))
    show = res if "--all" in sys.argv else res[:40]
    for r in show:
        m = r["mix"]
        print(f"{r['loop']:>10s} d{r['depth']} blk {r['blocks']:3d} instr {r['instructions']:5d} pk {m.get('valu_packed', 0):4d} "
              f"valu {m.get('valu', 0):4d} rdl {m.get('readlane', 0):3d} wrl {m.get('writelane', 0):3d} salu {m.get('salu', 0):4d} "
              f"nop {m.get('s_nop', 0):3d}/{r['s_nop_wait_states']:3d} lds {m.get('lds', 0):3d} br {m.get('branch', 0):3d} "
              f"vmem {m.get('vmem', 0):3d} -> {r['issue_cycles_lone_wave']} cyc")
    if "--json" in sys.argv:
        print(json.dumps(res))


if __name__ == "__main__":
    main()
