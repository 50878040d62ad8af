import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "fp-mash_amd")]
order = sys.argv[1]
import numpy as np
if order == "torch_first":
    import torch
    torch.cuda.set_device(0)
    t = torch.arange(1000, device="cuda:0", dtype=torch.int64)
    print("torch ok", int(t.sum()))
    import fpmash
    ctx = fpmash.Context(0)
    b = fpmash.DeviceBuffer.from_array(ctx, np.arange(1000, dtype=np.int64))
    print("fpmash ok", int(b.to_array(np.int64, 1000).sum()))
    # cross-runtime copy: torch tensor -> fpmash buffer
    L = fpmash.lib()
    rc = L.fpm_memcpy_d2d(ctx.h, b.ptr, t.data_ptr(), 8000, None)
    ctx.synchronize()
    print("d2d rc", rc, int(b.to_array(np.int64, 1000).sum()))
else:
    import fpmash
    ctx = fpmash.Context(0)
    print("fpmash ok")
    import torch
    print("torch avail", torch.cuda.is_available())
