set -o pipefail
# rocprofv3 kernel trace of the fwd + fa2_backward step at B2_H8_S512_D64 (tools/kbench.py stepb):
# per-kernel durations and the gaps between them -> gpurun_out/p${TAG:-512}/gaps.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p${TAG:-512}
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p${TAG:-512} -o run -- python3 tools/kbench.py --shape ${SHAPE:-2,8,512,64} --kernel stepb --do ones --rounds 2 --iters 20 > gpurun_out/p${TAG:-512}/kb.log 2>&1 || exit $?
f=$(find gpurun_out/p${TAG:-512} -name "*kernel_trace.csv" | head -1)
python3 - "$f" > gpurun_out/p${TAG:-512}/gaps.txt <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
rows=[r for r in rows if "fa2" in r["Kernel_Name"] or "delta" in r["Kernel_Name"]]
last=rows[-60:]
prev=None
for r in last:
    s,e=int(r["Start_Timestamp"]),int(r["End_Timestamp"])
    gap=(s-prev)/1000 if prev else 0
    print(f"{r['Kernel_Name'][:70]:70s} dur {(e-s)/1000:7.2f} us gap {gap:6.2f} grid {r.get('Grid_Size','')} wg {r.get('Workgroup_Size','')} lds {r.get('LDS_Block_Size', r.get('Lds_Size',''))}")
    prev=e
PY
