import csv, sys, re, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "ntt_pass" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = collections.defaultdict(list)
for i, r in enumerate(rows):
    by[i % 3].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(by.items()):
    print("pass", k, "ms", [round(x, 4) for x in v], "grid", rows[k]["Grid_Size_X"], "vgpr", rows[k]["VGPR_Count"], "lds", rows[k]["LDS_Block_Size"])
