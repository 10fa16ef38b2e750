"""Average kernel-trace duration of one kernel per consecutive chunk of launches
(one chunk per A/B pass of a microbenchmark run under rocprofv3).

    python tools/split_trace.py <trace dir> <kernel substring> <launches per chunk>
"""
import csv
import glob
import os
import sys


def main():
    d, name, chunk = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if name in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    for i in range(0, len(rows), chunk):
        part = rows[i:i + chunk]
        durs = sorted(e - s for s, e in part)
        print(f"chunk {i // chunk}: {len(part)} launches, avg {sum(durs) / len(durs) / 1e3:.2f} us, "
              f"med {durs[len(durs) // 2] / 1e3:.2f} us")


if __name__ == "__main__":
    main()
