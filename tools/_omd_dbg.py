import torch, json, sys
sys.path.insert(0, '.')
from nvidia_terraform_modules_amd import ops
for (m,n,k) in [(5000,4104,768),(4608,4608,768),(4608,4360,768),(5000,4608,768)]:
    a = ops.fill_uniform_(torch.empty((m,k),dtype=torch.bfloat16,device='cuda'),1)
    b = ops.fill_uniform_(torch.empty((n,k),dtype=torch.bfloat16,device='cuda'),2)
    c1 = ops.gemm_bf16(a,b,variant='pingpong8cm')
    c2 = torch.full((m,n),7.0,dtype=torch.bfloat16,device='cuda')
    ops.gemm_bf16(a,b,c2,variant='pingpong8omd')
    bad = (c1 != c2)
    nb = int(bad.sum())
    out = {"shape":[m,n,k],"bad":nb}
    if nb:
        idx = bad.nonzero()
        r = idx[:,0]; cc = idx[:,1]
        out.update(rows=[int(r.min()),int(r.max())], cols=[int(cc.min()),int(cc.max())])
        tiles = sorted(set((int(x)//256, int(y)//256) for x,y in idx[:20000].tolist()))
        out["tiles"] = tiles[:40]; out["ntiles_bad"]=len(tiles)
        out["untouched_7"] = int((c2[bad]==7.0).sum())
        out["rowmod"] = sorted(set(int(x)%256//16 for x in r[:5000].tolist()))
        out["colmod"] = sorted(set(int(y)%256//32 for y in cc[:5000].tolist()))
    print(json.dumps(out), flush=True)
