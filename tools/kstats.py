"""Print Name, Calls, Average ms of a rocprofv3 kernel_stats.csv (short names)."""
import csv
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        n = r["Name"].split("(")[0].replace("void ", "").replace("pzk::", "")
        print("  %-32s %4s %9.3f ms  total %9.3f ms" % (n, r["Calls"], float(r["AverageNs"]) / 1e6,
                                                     float(r["TotalDurationNs"]) / 1e6))
