import json, sys
d=json.load(open(sys.argv[1])); c=d["concurrent_native"]
print(sys.argv[1], "lone", round(d["p50_latency_us"],1), "resident", round(d["p50_latency_resident_us"],1))
for k,v in c.items():
    if isinstance(v, dict) and k.startswith("resident"): print(" ", k, round(v["calls_per_s"]), round(v.get("mean_call_us"),1))
