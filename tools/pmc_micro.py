"""Per-dispatch SQ counters of the micro-benchmarks (velbench / posbench) from a rocprofv3 --pmc
counter_collection.csv: python tools/pmc_micro.py CSV KIND

KIND velbench: the dispatches follow tools/velbench.py's order (blocks 1, 1024, 4096; the islands of
its list, each measured then warmed); posbench: tools/posbench.py's (blocks 1, 1024).  Prints, for the
one-wave (blocks 1) dispatches, the executed instructions per contact update (velbench: 180 sweeps x
nc) or per pass (posbench), so cycles per update / (4 x instructions) says how close a chain is to
its issue floor (MI355X_MICROARCH.md: one wave issues one instruction per 4 cycles)."""
import csv
import sys
from collections import OrderedDict


def dispatches(path, kernel):
    d = OrderedDict()
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel not in row["Kernel_Name"]:
                continue
            k = int(row["Dispatch_Id"])
            e = d.setdefault(k, {"grid": int(row["Grid_Size"])})
            e[row["Counter_Name"]] = float(row["Counter_Value"])
    return list(d.values())


def main():
    path, kind = sys.argv[1], sys.argv[2]
    if kind == "velbench":
        ds = dispatches(path, "k_velbench")
        combos = [(1, 1), (1, 2), (2, 2), (3, 2), (4, 2), (6, 2), (104, 2), (106, 2)]
        one = [d for d in ds if d["grid"] == 64]
        for i, (nc, pc) in enumerate(combos):
            if 2 * i >= len(one):
                break
            d = one[2 * i]
            upd = 180 * (nc % 100)
            print(f"velbench nc {nc} points {pc}: instructions per update {d.get('SQ_INSTS', 0) / upd:7.1f}  "
                  f"VALU {d.get('SQ_INSTS_VALU', 0) / upd:6.1f}  SALU {d.get('SQ_INSTS_SALU', 0) / upd:6.1f}  "
                  f"branch {d.get('SQ_INSTS_BRANCH', 0) / upd:5.1f}")
    else:
        ds = dispatches(path, "k_posbench")
        combos = [(1, 1), (1, 2), (2, 2), (3, 2), (4, 2), (3, 1)]
        one = [d for d in ds if d["grid"] == 64]
        for i, (nc, pc) in enumerate(combos):
            if 2 * i >= len(one):
                break
            d = one[2 * i]
            print(f"posbench nc {nc} points {pc}: instructions {d.get('SQ_INSTS', 0):9.0f}  VALU {d.get('SQ_INSTS_VALU', 0):8.0f}  "
                  f"SALU {d.get('SQ_INSTS_SALU', 0):8.0f}  branch {d.get('SQ_INSTS_BRANCH', 0):7.0f}  (divide by passes x nc x points)")


if __name__ == "__main__":
    main()
