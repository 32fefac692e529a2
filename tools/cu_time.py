import csv,collections,sys
rows=list(csv.DictReader(open(sys.argv[1])))
d=collections.OrderedDict()
for r in rows:
    e=d.setdefault(int(r['Dispatch_Id']),dict(r)); e[r['Counter_Name']]=float(r['Counter_Value'])
ds=sorted(d.values(), key=lambda e:int(e['Dispatch_Id']))
idx=[i for i,e in enumerate(ds) if e['Kernel_Name'].startswith('dbslmm_unpack')]
last=ds[idx[-2]:]
cap={'dbslmm_tchol_trailing3k16':16,'dbslmm_tchol_region':4,'dbslmm_tchol_panel':8,'dbslmm_gram_huge':8,'dbslmm_gram_big':8,
'dbslmm_gram_i8':32,'dbslmm_chol_large':4,'dbslmm_chol_cheb':8,'dbslmm_trsv_bwd':9,'dbslmm_trsv_fwd':9,'dbslmm_unpack_stats':32,'dbslmm_chol_small':8,'dbslmm_cheb_init':32}
agg=collections.defaultdict(lambda:[0,0.,0.])
clk=2.4e9
for e in last:
    n=e['Kernel_Name'].split('(')[0].replace('void ','').split('<')[0]
    if n not in cap: continue
    cu_ms=e['SQ_WAVE_CYCLES']*4/cap[n]/clk*1e3/256
    dur=(int(e['End_Timestamp'])-int(e['Start_Timestamp']))/1e6
    a=agg[n]; a[0]+=1; a[1]+=cu_ms; a[2]+=dur
tot=0
for k,a in sorted(agg.items(), key=lambda x:-x[1][1]):
    print(f"{k:28s} n={a[0]:4d} chip-ms(CU-time/256)={a[1]:7.2f}  serialized dur={a[2]:7.2f}")
    tot+=a[1]
print('total chip-ms %.2f'%tot)
