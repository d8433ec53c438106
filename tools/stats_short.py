"""Print name / calls / average us of a rocprofv3 kernel_stats.csv (names shortened)."""
import csv
import re
import sys

for row in csv.DictReader(open(sys.argv[1])):
    name = row["Name"].replace("phx::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)
    print(f"{name:60s} {int(row['Calls']):6d} {float(row['AverageNs'])/1000:9.2f} us  {float(row['Percentage']):6.2f}%")
