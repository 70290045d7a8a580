import time, torch
print("mem_get_info", torch.cuda.mem_get_info())
p = torch.cuda.get_device_properties(0)
print("props", p.name, p.total_memory, p.multi_processor_count, getattr(p, "gcnArchName", ""))
x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
print("after 4GiB mem_get_info", torch.cuda.mem_get_info())
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(3): a @ a
torch.cuda.synchronize(); t = time.time()
for _ in range(20): a @ a
torch.cuda.synchronize(); dt = (time.time() - t) / 20
print("matmul8k ms %.3f TFLOPs %.1f" % (dt * 1e3, 2 * 8192**3 / dt / 1e12))
