"""Per step of each traced process (tools/r05_modes.sh): the rest unpack's end, the lead chain's first region
and the host times of the hipGraphLaunch calls (HIP runtime trace) -- the step modes vs the host
side.  python tools/step_modes_api.py"""
import csv, sys
for i in (1,2,3,4):
    base=f'gpurun_out/r05modes/p{i}'
    k=list(csv.DictReader(open(base+'/run_kernel_trace.csv'))); k.sort(key=lambda r:int(r['Start_Timestamp']))
    a=list(csv.DictReader(open(base+'/run_hip_api_trace.csv'))); a.sort(key=lambda r:int(r['Start_Timestamp']))
    nm=lambda r:r['Kernel_Name'].replace('void ','').split('(')[0]
    idx=[j for j,r in enumerate(k) if nm(r).startswith('dbslmm_unpack')]
    gl=[r for r in a if r['Function']=='hipGraphLaunch']
    print(f'p{i}: graph launches {len(gl)}')
    for s in range(0,len(idx)-1,2):
        j=idx[s]; t0=int(k[j]['Start_Timestamp'])
        ue=int(k[idx[s+1]]['End_Timestamp'])
        fr=next((r for r in k[j:] if nm(r)=='dbslmm_tchol_region'),None)
        # host: graph launches after this step's first unpack start - host calls happen before; find launches within [t0-5ms, t0+20ms]
        g=[r for r in gl if t0-20_000_000 < int(r['Start_Timestamp']) < t0+30_000_000]
        gs=' '.join('%.2f..%.2f'%((int(r['Start_Timestamp'])-t0)/1e6,(int(r['End_Timestamp'])-t0)/1e6) for r in g[:3])
        # host time of the unpack launch call
        print('  step %d unpack_end %.2f first_region %.2f  graphLaunch(host) %s'%(s//2,(ue-t0)/1e6,(int(fr['Start_Timestamp'])-t0)/1e6 if fr else -1, gs))
