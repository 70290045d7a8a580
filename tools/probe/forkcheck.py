import os, sys, subprocess
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from amdvgpu.shim.launcher import vgpu_env, apply_contract, cleanup_region
c = vgpu_env(mem_limit=4 << 30)
code = r"""
import os, torch
a = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
pid = os.fork()
if pid == 0:
    os._exit(0 if sum(range(10)) == 45 else 1)
_, st = os.waitpid(pid, 0)
b = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
k = torch.ones(1 << 20, device="cuda").sum().item()  # kernel launches through the gates
torch.cuda.synchronize()
free, total = torch.cuda.mem_get_info()
print("forkcheck", os.WEXITSTATUS(st), total == (4 << 30), k == float(1 << 20), flush=True)
"""
r = subprocess.run([sys.executable, "-c", code], env=apply_contract(c), capture_output=True, text=True, timeout=60)
cleanup_region(c)
print(r.stdout.strip(), r.returncode, r.stderr[-500:])
sys.exit(r.returncode)
