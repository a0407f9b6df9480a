"""Summarise tools/pmc_dense.sh output (SQ / GRBM counters per dispatch of tools/phase_timing.py) into JSON.

usage: python3 tools/pmc_sq_summary.py gpurun_out/pmc_dense.txt profiles/r03/train/pmc_sq_dense.json

Per kernel (dispatches of one kernel averaged): mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs
x 1024 SIMDs); issued FLOP = SQ_INSTS_MFMA x 16384 (16x16x32 f16/bf16 MFMA: the Linears' and aggregations'
instruction; the few f32 16x16x4 MFMAs of the 8-input embeddings are counted at the same weight, an upper
bound); wave-time shares from SQ_WAVE_CYCLES; LDS bank conflicts per LDS-active cycle."""
import collections
import json
import sys


def main(src, dst):
    per = collections.OrderedDict()
    for line in open(src):
        tok = line.split()
        if len(tok) < 3 or not tok[0].isdigit() or "mpnn" not in line:
            continue
        name = " ".join(t for t in tok[1:] if "=" not in t).replace("void ", "").replace("eco::", "")
        cs = dict((t.split("=")[0], float(t.split("=")[1])) for t in tok[1:] if "=" in t)
        per.setdefault(name, []).append(cs)
    out = {"source": f"rocprofv3 --pmc (two SQ/GRBM passes) over tools/phase_timing.py (tools/pmc_dense.sh): {src}",
           "notes": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": {}}
    for name, rows in per.items():
        keys = set().union(*rows)
        c = {k: sum(r.get(k, 0.0) for r in rows) / len(rows) for k in sorted(keys)}
        e = {"dispatches": len(rows), "counters": c}
        if c.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        e["issued_mfma_flop"] = c.get("SQ_INSTS_MFMA", 0.0) * 16384
        if c.get("SQ_WAVE_CYCLES"):
            for k, s in (("SQ_WAIT_ANY", "wait_any_share"), ("SQ_WAIT_INST_ANY", "wait_inst_share"),
                         ("SQ_ACTIVE_INST_ANY", "active_share")):
                if k in c:
                    e[s] = c[k] / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_per_lds_active"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        out["kernels"][name] = e
        print(f"{name:50s} n={len(rows)} mfma_busy={e.get('mfma_busy', 0):.3f} "
              f"wait={e.get('wait_any_share', 0):.3f} active={e.get('active_share', 0):.3f}")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
