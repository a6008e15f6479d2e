import csv, statistics as st, sys
rows=[list(map(int,r)) for r in csv.reader(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/mapcyc.csv')) if int(r[6])>0]
for i,name in enumerate(["wait","byte+list","passA","passB"]):
    v=[r[1+i] for r in rows]; print("%-10s med %.0f kcyc  (per row %.0f cyc)"%(name, st.median(v)/1e3, st.median(r[1+i]/r[6] for r in rows)))
print("rows/wave med", st.median(r[6] for r in rows), "misses/row", round(st.median(r[5]/r[6] for r in rows),1))
print("total med kcyc", st.median(sum(r[1:5]) for r in rows)/1e3)
