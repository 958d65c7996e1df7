import sqlite3, sys
db=sqlite3.connect(sys.argv[1])
rows=list(db.execute("select name,start,end,queue_id from kernels order by start"))
# steps bounded by adam_dev_kernel ends
marks=[i for i,r in enumerate(rows) if 'adam_dev_kernel' in r[0]]
# take the last full step between the last two adam markers
a,b=marks[-3],marks[-2]
step=rows[a+1:b+1]
t0=rows[a][2]; t1=step[-1][2]
print("step wall us", (t1-t0)/1e3, "kernels", len(step), "sum dur us", sum(r[2]-r[1] for r in step)/1e3)
# busy union and gaps
ev=sorted((r[1],r[2]) for r in step)
busy=0; cur_s,cur_e=ev[0]; gaps=[]
prev_end=t0
for s,e in ev:
    if s>cur_e:
        busy+=cur_e-cur_s; gaps.append((s-cur_e,cur_e)); cur_s,cur_e=s,e
    else: cur_e=max(cur_e,e)
busy+=cur_e-cur_s
print("busy union us", busy/1e3, "idle us", (t1-t0-busy)/1e3, "n gaps", len(gaps))
# concurrency: time with >=2 kernels
qs={}
for r in step: qs[r[3]]=qs.get(r[3],0)+1
print("queues", qs)
# longest idle gaps and the kernel after
gaps.sort(reverse=True)
idx={r[1]:r for r in step}
for g,e in gaps[:12]:
    nxt=min((r for r in step if r[1]>=e+g-1), key=lambda r:r[1])
    print(f"  gap {g/1e3:6.2f} us before {nxt[0][:70]}")
# histogram of gaps
import collections
h=collections.Counter(min(int(g/1e3),20) for g,_ in gaps)
print(sorted(h.items()))
