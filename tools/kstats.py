"""Print a rocprofv3 kernel_stats.csv summary: python tools/kstats.py DIR"""
import csv, glob, sys
for p in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        print("%-44s %5s %12.1f us %6.2f%%" % (r["Name"][:44], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
