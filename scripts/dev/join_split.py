"""Development: build vs probe split of the 2^28 counting join (per-workgroup ticks)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "../../sgxv2-analytical-query-processing-benchmarks_amd/python")]
import torch
import sgxamd
n = 1 << 28
torch.cuda.set_device(0)
s = torch.cuda.current_stream().cuda_stream
sgxamd.set_stream(s)
sgxamd.timing_enable(True)
R = torch.empty(n, dtype=torch.int64, device="cuda"); S = torch.empty(n, dtype=torch.int64, device="cuda")
sgxamd.gen_pk_dev(R, n, 0, n, 11111, s); sgxamd.gen_fk_dev(S, n, 0, n, 22222, s); torch.cuda.synchronize()
for i in range(3):
    r = sgxamd.rho_join(R, n, S, n)
st = r.stats
print({k: round(st[k], 4) for k in ("ms_join", "ms_build", "ms_probe")}, "tasks", st["num_tasks"], "max_part_r", st["max_part_r"])
