"""Per-kernel HBM traffic from rocprofv3 --pmc counter CSVs (one pass per counter):
    python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json
FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch.  gfx950
correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
(16 B/lane) coalesced reads, LDS-DMA included -> x2; WRITE_SIZE is exact for 16 B/lane stores.
Output: {kernel symbol: {dispatches, fetch_bytes, write_bytes, traffic_bytes}} averaged per launch."""
import collections
import csv
import glob
import json
import sys


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out[k] = dict(dispatches=max(len(f), len(w)), fetch_bytes=fb, write_bytes=wb,
                      traffic_bytes=(fb or 0.0) + (wb or 0.0))
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    top = sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes"] * kv[1]["dispatches"])[:12]
    for k, v in top:
        print(f"{v['traffic_bytes'] / 1e6:10.2f} MB/launch x{v['dispatches']:5d}  {k[:100]}")


if __name__ == "__main__":
    main()
