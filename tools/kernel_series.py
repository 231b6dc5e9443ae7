import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sent = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
a, b = sent[-2], sent[-1]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[a + 1:b]]
print("n", len(d), "first 10:", [round(x, 1) for x in d[:10]])
for i in range(0, len(d), 40):
    c = d[i:i + 40]
    print(f"launches {i}-{i + len(c) - 1}: mean {sum(c) / len(c):.2f} us")
# before the region: warm-up launches
pre = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[:a] if "digest_line" in r["Kernel_Name"]]
print("pre-region digest launches:", len(pre), "last 12:", [round(x, 1) for x in pre[-12:]])
gaps = []
for i in range(max(0, a - 15), a + 1):
    gaps.append(round((int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3, 1))
print("gaps (us) before the region:", gaps, [rows[i]["Kernel_Name"][:25] for i in range(max(0, a - 15), a + 1)][-6:])
