import csv,glob,sys
p=glob.glob(sys.argv[1]+'/*/*kernel_trace.csv')[0]
rows=[]
for r in csv.DictReader(open(p)):
    n=r["Kernel_Name"].split("(")[0].replace("void ","").split("<")[0].split("::")[-1]
    rows.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),n))
rows.sort()
idx=[i for i,r in enumerate(rows) if r[2]=="tr_chunk_info"]
i0=idx[int(sys.argv[2])]; i1=idx[int(sys.argv[2])+1] if len(idx)>int(sys.argv[2])+1 else len(rows)
t0=rows[i0][0]; last=t0
for s,e,k in rows[i0:min(i1,i0+int(sys.argv[3]))]:
    print("%9.1f gap %7.1f dur %7.1f %s"%((s-t0)/1e3,(s-last)/1e3,(e-s)/1e3,k))
    last=max(last,e)
