import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
q = next(r["Queue_Id"] for r in rows if r["Kernel_Name"].startswith("tick"))
segs, cur = [], []
for r in rows:
    if r["Queue_Id"] != q:
        continue
    if r["Kernel_Name"].startswith("spin") and len(cur) >= 300:
        segs.append(cur)
        cur = []
    elif r["Kernel_Name"].startswith("tick"):
        cur.append(r)
segs.append(cur)
for m, s in enumerate(segs):
    g = sorted((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000 for a, b in zip(s, s[1:]))
    if g:
        print(f"segment {m}: {len(s)} ticks, median gap {g[len(g) // 2]:.2f} us, p90 {g[9 * len(g) // 10]:.2f}")
