"""Kernel and copy totals of the last migrating batch in a rocprofv3 SQLite trace (tools/dev/r06p.sh,
r06q.sh): the window from the last gap before the last 8 mig_start launches to the trace's end.
  python tools/trace_window.py <results.db>"""
import sqlite3, collections, sys
c=sqlite3.connect(sys.argv[1])
ks=c.execute("select name,start,end,queue_id,stream_id from kernels order by start").fetchall()
ms=c.execute("select name,start,end,size,queue_id from memory_copies order by start").fetchall()
starts=[k[1] for k in ks if 'mig_start(' in k[0]]
print('mig_start launches', len(starts))
b0=starts[-8]; 
# batch begins somewhat before mig_start (resolve, route); take from previous batch end: last kernel ending before the 8th-last mig_start minus gap
prev=[k for k in ks if k[2] < starts[-16]] if len(starts)>=16 else []
# choose window: from the resolve kernel preceding: find first kernel after the last batch's predecessor's final kernel
ends_before=[k[2] for k in ks if k[1] < b0]
# find largest gap before b0 within 50ms
cand=[k for k in ks if b0-50e6 < k[1] < b0]
gaps=[(cand[i+1][1]-cand[i][2], cand[i+1][1]) for i in range(len(cand)-1)]
w0=max(gaps)[1] if gaps else b0
w1=max(k[2] for k in ks)
print('window ms', (w1-w0)/1e6)
agg=collections.defaultdict(lambda:[0,0.0])
for n,s,e,q,st in ks:
    if s>=w0 and e<=w1:
        nm=n.replace('keto::(anonymous namespace)::','')[:50]; agg[nm][0]+=1; agg[nm][1]+=(e-s)/1e6
tot=0
for nm,(cnt,t) in sorted(agg.items(), key=lambda x:-x[1][1]): print(f"{t:8.3f} ms {cnt:5d} {nm}"); tot+=t
print('kernel sum', round(tot,3))
magg=collections.defaultdict(lambda:[0,0.0,0])
for n,s,e,sz,q in ms:
    if s>=w0 and e<=w1: magg[n][0]+=1; magg[n][1]+=(e-s)/1e6; magg[n][2]+=sz
for n,(cnt,t,sz) in magg.items(): print(f"copy {n}: {cnt} copies {t:.3f} ms {sz/1e6:.1f} MB")
# busy union
iv=sorted([(s,e) for _,s,e,_,_ in ks if s>=w0 and e<=w1]+[(s,e) for _,s,e,_,_ in ms if s>=w0 and e<=w1])
u=0; cs,ce=None,None
for s,e in iv:
    if cs is None: cs,ce=s,e
    elif s>ce: u+=ce-cs; cs,ce=s,e
    else: ce=max(ce,e)
if cs is not None: u+=ce-cs
print('busy union ms', u/1e6)
