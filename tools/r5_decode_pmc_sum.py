"""Summarise tools/r5_decode_pmc.sh's two SQ passes per kernel family (runs on the GPU box)."""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k in sorted(tot):
    v = {c: tot[k][c] / cnt[k][c] for c in tot[k]}
    g = lambda c: v.get(c, float("nan"))  # noqa: E731
    wc = g("SQ_WAVE_CYCLES")
    print(k, "dispatches", cnt[k].get("SQ_WAVE_CYCLES", 0))
    print(f"   wait {g('SQ_WAIT_ANY')/wc:.3f} wait_inst {g('SQ_WAIT_INST_ANY')/wc:.3f} valu_active {g('SQ_ACTIVE_INST_VALU')/wc:.3f}"
          f" lds_active {g('SQ_ACTIVE_INST_LDS')/wc:.3f} any_active {g('SQ_ACTIVE_INST_ANY')/wc:.3f} misc {g('SQ_ACTIVE_INST_MISC')/wc:.3f}"
          f" valu/mfma {g('SQ_INSTS_VALU')/max(1, g('SQ_INSTS_MFMA')):.2f} valu/vmem {g('SQ_INSTS_VALU')/max(1, g('SQ_INSTS_VMEM_RD')):.2f}"
          f" salu/vmem {g('SQ_INSTS_SALU')/max(1, g('SQ_INSTS_VMEM_RD')):.2f} vmem_cyc/inst {g('SQ_INST_CYCLES_VMEM_RD')/max(1, g('SQ_INSTS_VMEM_RD')):.1f}"
          f" mfma_busy/cu_cycles {g('SQ_VALU_MFMA_BUSY_CYCLES')/(g('GRBM_GUI_ACTIVE')/8*1024):.3f} waves {g('SQ_WAVES'):.0f} wave_cycles {wc:.0f}")
