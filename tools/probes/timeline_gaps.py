import gzip,csv,sys
tag=sys.argv[1]
rows=list(csv.DictReader(gzip.open(f'/root/repo/gpurun_out/{tag}/kernel_trace.csv.gz','rt')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
names=[r['Kernel_Name'] for r in rows]
idx=[i for i,n in enumerate(names) if 'stem_wgrad_kernel' in n]
for k in range(len(idx)-6, len(idx)-1):
    seq=rows[idx[k]:idx[k+1]]
    end=int(seq[0]['End_Timestamp']); prevn=''; big=[]; tot=0
    for r in seq[1:]:
        s=int(r['Start_Timestamp'])
        if s-end>15000:
            tot+=(s-end)/1e3
            if s-end>300000: big.append((round((s-end)/1e3,1), prevn, r['Kernel_Name'].split('(')[0][:40]))
        if int(r['End_Timestamp'])>end: end=int(r['End_Timestamp']); prevn=r['Kernel_Name'].split('(')[0][:40]
    span=(int(seq[-1]['End_Timestamp'])-int(seq[0]['Start_Timestamp']))/1e6
    print(f"step {k}: span {span:.2f} ms, gaps>15us {tot:.0f} us", big)
