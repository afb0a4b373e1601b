"""Key numbers of a bench.py log's JSON line (the last one): python tools/_bench_summary.py LOG"""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]
d = json.loads(line)
e = d["extras"]
print("K1", d["roofline"]["kernel_ms"], d["roofline"]["frac"], "placements", d["roofline"]["placement"]["tried_ms"])
print("pipeline", d["pipeline"]["gpu_ms_per_call"], d["pipeline"]["frac"],
      "planes", e["pipeline_frame_planes"]["gpu_ms_per_call"], e["pipeline_frame_planes"]["frac"])
print("loop", e["device_frame_loop"]["ms_per_batch"], e["device_frame_loop"]["stage_ms"])
print("sgbm", e["sgbm_disparity"]["us_per_frame"], e["sgbm_disparity"].get("placement", {}).get("tried_ms"),
      e["sgbm_disparity"].get("placement", {}).get("kept"))
print("parity", d["parity"]["pass"], "latency_us", d.get("latency_1frame_us"))
