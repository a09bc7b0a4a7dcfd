"""HBM traffic of k_step per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md prescribes (FETCH_SIZE x 2 on gfx950; both counters in KiB).
    python tools/traffic.py <fetch_dir> <write_dir> <env_id> <lanes> [profiles/pmc_traffic.json]
Merges {env_id: {...}} into the json file bench.py reads for roofline.traffic."""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kname="k_step"):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kname} under {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, env, lanes = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    fetch_kib, nf = per_dispatch(fdir, "FETCH_SIZE")
    write_kib, nw = per_dispatch(wdir, "WRITE_SIZE")
    fetch_b, write_b = 2.0 * fetch_kib * 1024.0, write_kib * 1024.0
    d = {}
    if os.path.exists(out):
        d = json.load(open(out))
    d[str(env)] = {"lanes": lanes, "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
                   "hbm_bytes_per_launch": fetch_b + write_b, "dispatches": [nf, nw],
                   "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes, k_step average; "
                             "FETCH_SIZE (KiB) x2 per MI355X_MICROARCH.md gfx950 correction"}
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(d[str(env)]))


if __name__ == "__main__":
    main()
