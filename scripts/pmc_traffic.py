"""HBM traffic per dispatch from the rocprofv3 --pmc passes of scripts/pmc.sh (FETCH_SIZE, WRITE_SIZE; one
counter per pass).  Corrections from MI355X_MICROARCH.md §HBM: both counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of 16-byte-per-lane streaming reads, so it is doubled.

    python3 scripts/pmc_traffic.py gpurun_out/pmc [precision]

Writes <root>/pmc_traffic_<precision>.json: {"kernels": {kernel: {fetch_bytes, write_bytes, hbm_bytes, dispatches}},
"scopes": {bench profiler scope: same}} - the scope table is what bench.py's roofline reads (every scope below is one
kernel instantiation with one launch shape, so its per-dispatch average is well defined)."""
import collections
import csv
import json
import os
import sys

# bench.py profiler scope -> substring of the demangled kernel name (rocprofv3 Kernel_Name)
SCOPES = {
    "fp32": {
        "f32_conv1_fwd": "k_conv1_fwd32<0, true>",   # one sample per block (round 6)
        "f32_conv1_fwd_big": "k_conv1_fwd32<1, false>",
        # row-list forwards (non-background rows + the background rows' side blocks)
        # (the training-batch and the chunk-batch conv2 forward are one instantiation (64 x 64 list tiles): one entry, the
        # average over both kinds of dispatch)
        "f32_conv2_fwd_big": "k_gemm32_side<qlx::q32::PConvFwdL<20, 20, 32, 4, 2, 9, 9, 64, 64, 64,",
        "f32_conv3_fwd": "k_gemm32_side<qlx::q32::PConvFwdL<9, 9, 64, 3, 1, 7, 7, 64, 32, 64,",
        "f32_conv3_fwd_big": "k_gemm32_side<qlx::q32::PConvFwdL<9, 9, 64, 3, 1, 7, 7, 64, 64, 64,",
        "f32_fc1_fwd": "k_gemm32<qlx::q32::PFc1FwdT<32, 32, 2, 2,",
        "f32_fc1_fwd_big": "k_gemm32<qlx::q32::PFc1FwdT<64, 128, 2, 2,",
        "f32_fc1_bwd": "k_gemm32_pair<qlx::q32::PFc1WgradT",
        "f32_conv3_bwd": "k_gemm32_pair<qlx::q32::PConvWgrad<9, 9",
        "f32_conv2_bwd": "k_gemm32_pair<qlx::q32::PConvWgrad<20, 20",
        "f32_conv1_wgrad": "k_conv1_wgrad32",
        "f32_norms": "k_wreduce32",
        "f32_head": "k_head32<3, 4>",
        "f32_wgrad_reduce": "k_wreduce32",
        "f32_adam": "k_update32",   # update schedule 2 (default): every variable's clip_by_norm + Adam in one launch
    },
    "bf16": {
        # rocprofv3 leaves these names mangled: k_trunk_fwd<store = true, ...> (training batches) / <false, ...>
        "trunk_fwd": "k_trunk_fwdILb1E",
        "trunk_fwd_nostore": "k_trunk_fwdILb0E",
        "trunk_bwd_data": "k_trunk_bwd_data",
        "conv1_wgrad": "k_conv1_wgrad",
        "conv23_wgrad": "k_conv23_wgrad",
        "fc1_bwd": "k_fc1_bwd",
        "fc1_fwd": "k_bgemm<qlx::qn::BGemmCfg<128, 64, 2, 2, false, true, 4",   # the training-batch forward (4 k splits)
        "wgrad_reduce": "k_slab_reduce3",
        "fc2_head": "k_fc2_train",
        "adam": "k_adam(",
    },
}


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for pas, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = os.path.join(root, pas, "c_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]][counter].append(float(r["Counter_Value"]))
    kernels = {}
    for k, c in vals.items():
        fb = 2.0 * 1024 * sum(c["FETCH_SIZE"]) / max(1, len(c["FETCH_SIZE"]))
        wb = 1024.0 * sum(c["WRITE_SIZE"]) / max(1, len(c["WRITE_SIZE"]))
        kernels[k] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb),
                      "dispatches": len(c["FETCH_SIZE"])}
    scopes = {}
    for scope, key in SCOPES[prec].items():
        hits = [v for k, v in kernels.items() if key in k]
        if len(hits) == 1:
            scopes[scope] = hits[0]
    out = os.path.join(root, f"pmc_traffic_{prec}.json")
    json.dump({"corrections": "FETCH_SIZE x2 (gfx950, 16 B/lane reads), KiB -> bytes", "precision": prec, "kernels": kernels,
               "scopes": scopes}, open(out, "w"), indent=1)
    print(json.dumps({k: v["hbm_bytes"] for k, v in scopes.items()}, indent=1))


if __name__ == "__main__":
    main()
