"""Summarise dev/ceiling_lab's JSON lines (gpurun_out/ceiling.jsonl, `bash dev/lab.sh ceiling`) into
profiles/<tag>_ceilings.json: the best copy / read / write rate per buffer size and policy, the keys
pass's write-stream floor (runs64), and the per-XCC copy rates -- set beside MI355X_MICROARCH.md's
6.29 TB/s float4 copy (DESIGN §3 "Ceilings").

    python dev/ceilings.py gpurun_out/ceiling.jsonl profiles/r05_ceilings.json
"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
rows = [json.loads(ln) for ln in open(src) if ln.startswith("{")]
rates = [r for r in rows if "TBs" in r]


def best(pred):
    xs = [r for r in rates if pred(r)]
    return max(xs, key=lambda r: r["TBs"]) if xs else None


def pick(r):
    return None if r is None else {k: r[k] for k in ("kind", "mode", "threads", "quads_per_thread", "grid_per_cu",
                                                     "nt_loads", "nt_stores", "ms", "TBs")}


out = {
    "source": "dev/ceiling_lab.hip (bash dev/lab.sh ceiling), one MI355X box, HIP events, mean of 10 launches",
    "guide": "MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec, 6.29 TB/s measured float4 copy (buffer size not stated)",
    "bytes": "read + write bytes of the launch (copy: 2 x buffer)",
    "copy_2x4GiB_best": pick(best(lambda r: r["kind"] == "copy" and r["mode"] in ("stride_big", "chunk"))),
    "copy_2x4GiB_best_default_policy": pick(best(lambda r: r["kind"] == "copy" and r["mode"] == "stride_big"
                                                 and not r["nt_loads"] and not r["nt_stores"])),
    "copy_2x4GiB_one_chunk_per_workgroup_best": pick(best(lambda r: r["kind"] == "copy" and r["mode"] == "chunk")),
    "copy_2x256MiB_best": pick(best(lambda r: r["kind"] == "copy" and r["mode"] == "stride_256MiB")),
    "read_4GiB_best": pick(best(lambda r: r["kind"] == "read")),
    "write_4GiB_best": pick(best(lambda r: r["kind"] == "write")),
    "keys_pass_write_stream_floor": pick(best(lambda r: r["kind"] == "runs64")),
    "copy_2x4GiB_all": [pick(r) for r in rates if r["kind"] == "copy" and r["mode"] == "stride_big"],
    "copy_2x256MiB_all": [pick(r) for r in rates if r["kind"] == "copy" and r["mode"] == "stride_256MiB"],
    "chunk_rates_by_xcc": [{k: r[k] for k in ("mode", "workgroups", "wall_us", "end_spread_us", "dur_us_min_med_max",
                                             "xcc_not_blockIdx_mod_8", "by_xcc")}
                           for r in rows if r.get("kind") == "chunk_rates"],
}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps({k: out[k] for k in ("copy_2x4GiB_best", "copy_2x256MiB_best", "read_4GiB_best", "write_4GiB_best",
                                      "keys_pass_write_stream_floor")}, indent=1))
