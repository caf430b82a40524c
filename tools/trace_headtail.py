"""Head / tail split of one C2 step from a rocprofv3 kernel trace: wall time and per-class busy
time of the iterations with separate merge launches (head) and with k_merge_tail (tail), and the
head's merge-phase wall; with LAST, the last LAST iterations (e.g. C2's 282 below 2^20 rows,
round 4's "tail") apart.  python tools/trace_headtail.py run_kernel_trace.csv [LAST]"""
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
its=[];cur=None
for r in rows:
    n=r["Kernel_Name"]
    if "k_project" in n and "fix" not in n:
        cur=[];its.append(cur)
    if cur is not None: cur.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),n.split('(')[0].replace('void ','').replace('klsh::','')))
its=its[1:]
def cls(n):
    for k in ["project","sort","runs","tail_local","small_screen","merge_tail","merge_small","merge_big","merge_huge","merge_long","compact"]:
        if k in n: return k
    return n[:20]
tail=[i for i,k in enumerate(its) if any('merge_tail' in x[2] for x in k)]
print("tail iterations",len(tail),"first",tail[0] if tail else None)
last=int(sys.argv[2]) if len(sys.argv)>2 else 0
groups=[("head",[i for i in range(len(its)) if i not in set(tail)]),("tail",tail)]
if last: groups+=[("tail-mid",[i for i in tail if i<len(its)-last]),("last%d"%last,list(range(len(its)-last,len(its))))]
for name,sel in groups:
    tot=0;busy=collections.Counter()
    for i in sel:
        k=its[i]
        if i+1<len(its): end=its[i+1][0][0]
        else: end=max(b for a,b,n in k if 'stamp' not in n and 'rocclr' not in n and 'gather' not in n)
        tot+=end-k[0][0]
        for a,b,n in k: busy[cls(n)]+=b-a
    print(name,len(sel),"wall ms %.2f"%(tot/1e6))
    for c,v in busy.most_common(): print("   %-14s %8.2f ms"%(c,v/1e6))
print("---- head merge-phase wall")
mw=0;pre=0;post=0
for i in range(len(its)):
    if i in set(tail): continue
    k=its[i]
    m=[(a,b) for a,b,n in k if 'merge' in n]
    s=min(a for a,b in m); e=max(b for a,b in m)
    mw+=e-s; pre+=s-k[0][0]
    nxt=its[i+1][0][0]
    post+=nxt-e
print("merge wall %.2f  pre-merge %.2f  post-merge(compact+gap) %.2f"%(mw/1e6,pre/1e6,post/1e6))
