import torch, time
dev="cuda"
print(torch.cuda.get_device_properties(0).gcnArchName)
for dt in (torch.float8_e4m3fn, torch.float8_e4m3fnuz):
    try:
        M,N,K=256,4096,4096
        a=torch.randn(M,K,device=dev).to(dt); b=torch.randn(N,K,device=dev).to(dt)
        sa=torch.ones(M,1,device=dev); sb=torch.ones(1,N,device=dev)
        for name,(x,y) in {"tensor":(torch.tensor(1.0,device=dev),torch.tensor(1.0,device=dev)),"rowwise":(sa,sb)}.items():
            try:
                o=torch._scaled_mm(a,b.t(),scale_a=x,scale_b=y,out_dtype=torch.bfloat16)
                torch.cuda.synchronize()
                t=time.perf_counter()
                for _ in range(50): o=torch._scaled_mm(a,b.t(),scale_a=x,scale_b=y,out_dtype=torch.bfloat16)
                torch.cuda.synchronize()
                us=(time.perf_counter()-t)/50*1e6
                print(dt,name,"ok",o.shape, f"{us:.1f}us")
            except Exception as e: print(dt,name,"FAIL",str(e)[:200])
    except Exception as e: print(dt,"FAIL",str(e)[:200])
