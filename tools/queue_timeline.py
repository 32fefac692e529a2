import csv,collections,sys
t=list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda r:int(r["Start_Timestamp"]))
idx=[i for i,r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_unpack")]
last=t[idx[-2]:]
t0=int(last[0]["Start_Timestamp"])
by=collections.defaultdict(lambda: collections.defaultdict(lambda:[1e18,0,0,0.0]))
for r in last:
    k=r["Kernel_Name"].split("(")[0].replace("void ","").split("<")[0]
    s=(int(r["Start_Timestamp"])-t0)/1e3; e=(int(r["End_Timestamp"])-t0)/1e3
    a=by[r["Queue_Id"]][k]; a[0]=min(a[0],s); a[1]=max(a[1],e); a[2]+=1; a[3]+=e-s
for q in sorted(by):
    for k,a in sorted(by[q].items(), key=lambda x:x[1][0]):
        print(f"q{q} {k:28s} n={a[2]:3d} {a[0]/1e3:7.2f}-{a[1]/1e3:7.2f} ms  busy {a[3]/1e3:6.2f}")
