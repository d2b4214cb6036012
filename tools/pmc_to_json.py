"""Turn FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc.sh) into the per-launch HBM traffic record that
bench.py reports as roofline.traffic.

Corrections per MI355X_MICROARCH.md (HBM/rocprofv3 section): the counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores. The infer kernel reads the 60-B queries with
16-B loads and writes 12-B results with 4/8/16-B stores, so the write figure is an estimate.

    python tools/pmc_to_json.py gpurun_out/pmc_bench infer_kernel profiles/pmc_infer_r01.json
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import load  # noqa: E402


def main():
    d, filt, out = Path(sys.argv[1]), sys.argv[2], Path(sys.argv[3])
    per = load(d)
    ks = [k for k in per if filt in k]
    if len(ks) != 1:
        raise SystemExit(f"expected one kernel matching {filt!r}, got {ks}")
    cs = per[ks[0]]
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    fetch = mean["FETCH_SIZE"] * 1024 * 2
    write = mean["WRITE_SIZE"] * 1024
    rec = {"kernel": ks[0], "dispatches": {c: len(v) for c, v in cs.items()},
           "FETCH_SIZE_KiB": mean["FETCH_SIZE"], "WRITE_SIZE_KiB": mean["WRITE_SIZE"],
           "read_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "correction": "FETCH_SIZE x1024 x2 (gfx950 wide-read halving), WRITE_SIZE x1024"}
    out.write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
