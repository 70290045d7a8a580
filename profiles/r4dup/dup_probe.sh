cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dup
for v in "ROCR_VISIBLE_DEVICES=0,0" "HIP_VISIBLE_DEVICES=0,0"; do
  echo "== $v" >> gpurun_out/dup/out.txt
  env $v timeout -k 5 90 python -c "
import torch
n = torch.cuda.device_count()
print('count', n)
if n > 1:
    a = torch.ones(1 << 20, device='cuda:0'); b = torch.ones(1 << 20, device='cuda:1')
    torch.cuda.synchronize(0); torch.cuda.synchronize(1)
    print('props', [torch.cuda.get_device_properties(i).name for i in range(n)], float(a.sum() + b.sum().to('cuda:0')))
" >> gpurun_out/dup/out.txt 2>&1
  echo "rc=$?" >> gpurun_out/dup/out.txt
done
