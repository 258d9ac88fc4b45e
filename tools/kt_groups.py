import csv,collections,statistics as st,sys
rows=list(csv.DictReader(open(sys.argv[1])))
g=collections.defaultdict(list)
for r in rows:
    n=r["Kernel_Name"]
    short=n.split("(anonymous namespace)::")[-1].split("(")[0][:45] if "anonymous" in n else n[:45]
    g[(short, r["Grid_Size_X"], r["Grid_Size_Z"])].append((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000)
for k,v in sorted(g.items(), key=lambda kv:-len(kv[1]))[:5]:
    v=sorted(v); print(len(v), k, "p10 %.2f p25 %.2f med %.2f p75 %.2f"%(v[len(v)//10],v[len(v)//4],v[len(v)//2],v[3*len(v)//4]))
