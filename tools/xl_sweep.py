import os, sys, torch
sys.path.insert(0, os.getcwd())
from distributed_model_parallel_amd import _native
C = _native.require("x")
def timeit(fn, iters=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b)/iters
shapes=[(802816,128,1152),(200704,256,2304),(50176,512,4608),(200704,1024,256),(3211264,64,576),(12845056,64,256)]
for M,N,K in shapes:
    a=torch.rand(M,K,device='cuda',dtype=torch.bfloat16)*2-1
    b=torch.rand(N,K,device='cuda',dtype=torch.bfloat16)*2-1
    res={}
    res['nt']=timeit(lambda: C.gemm_nt(a,b))
    res['blaslt']=timeit(lambda: a@b.t())
    for bn in (128,256):
        for pipe in (1,6):
            for gm in (1,4,8):
                if N<bn and bn==256: continue
                C.set_gemm_xl_bn(bn,pipe,gm)
                res[f'xl{bn}p{pipe}g{gm}']=timeit(lambda: C.gemm_xl(a,b))
    C.set_gemm_xl_bn(0,1,0)
    best=min(res,key=res.get)
    print(M,N,K,' '.join(f'{k}={v:.3f}' for k,v in res.items()),'BEST',best,flush=True)
    del a,b; torch.cuda.empty_cache()
