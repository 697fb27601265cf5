"""Median times of the binning kernels after k_bin_count ends (one forward at a time) in a rocprofv3 kernel-trace CSV."""
import csv,sys,statistics
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def short(n):
    for k in ('k_bin_count','k_bin_table','k_tile_start_apply','k_bin_scatter','k_tile_sort_wave','k_preprocess_colour','k_preprocess<'):
        if k in n: return k
    return None
seq=[(short(r['Kernel_Name']),int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in rows]
seq=[s for s in seq if s[0]]
out={}
for i,(n,s,e) in enumerate(seq):
    if n=='k_bin_count':
        d={}
        for m,s2,e2 in seq[i:i+8]:
            d.setdefault(m,(s2,e2))
        if 'k_bin_scatter' in d:
            ce=e
            for m in ('k_bin_table','k_tile_start_apply','k_bin_scatter'):
                out.setdefault(m+'_start',[]).append((d[m][0]-ce)/1e3)
                out.setdefault(m+'_end',[]).append((d[m][1]-ce)/1e3)
for k,v in out.items(): print(k, round(statistics.median(v),2))
