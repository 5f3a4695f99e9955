set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/attn_tcc
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/attn_tcc/p1 -- python3 $R/tools/attn_only.py > $R/gpurun_out/attn_tcc/p1.log 2>&1
echo p1=$?
python3 - <<'PY'
import csv,glob,os,collections
R=os.environ['GRAFT_REPO_ROOT']
for p in ['p1']:
    f=sorted(glob.glob(R+f'/gpurun_out/attn_tcc/{p}/*/*counter_collection.csv'))[-1]
    agg=collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        n=r['Kernel_Name']
        if 'fa' not in n: continue
        agg[n.split('(')[0][-30:]][r['Counter_Name']]+=float(r['Counter_Value'])
    for k,v in agg.items():
        h,m=v.get('TCC_HIT_sum',0),v.get('TCC_MISS_sum',0)
        print(k, {a:f"{b:.3e}" for a,b in v.items()}, 'hit%%=%.1f'%(100*h/max(1,h+m)))
PY
