import sys, os, json
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "../../sgxv2-analytical-query-processing-benchmarks_amd/python")]
import sgxamd as sgx
R, S = sgx.reference_relations(1 << 20, 1 << 20, selectivity=50)
res = sgx.rho_join_multi(R, len(R), S, len(S), 4, transport="rehearsal", radix_bits=10, passes=2)
d = res.stats
print(json.dumps({k: v for k, v in d.items() if k != "local"}))
print(json.dumps(d["local"]))
r1 = sgx.rho_join(R, len(R), S, len(S), radix_bits=10, passes=2)
print(json.dumps(r1.stats))
