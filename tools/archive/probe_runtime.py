"""Probe: can torch's bundled HIP runtime and /opt/rocm's runtime (our library) share a process?"""
import sys, ctypes, numpy as np
sys.path.insert(0, "orb-slam2-noted_amd/python")
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch cuda", torch.cuda.is_available(), flush=True)
    x = torch.arange(16, dtype=torch.uint8, device="cuda")
    import orbslam2_amd as amd
    print("amd devices", amd.device_count(), flush=True)
    ex = amd.BatchExtractor(500)
    img = np.random.default_rng(0).integers(0, 255, (480, 640), dtype=np.uint8)
    t = torch.from_numpy(img).cuda(); torch.cuda.synchronize()
    try:
        ex.reserve(640, 480, 1)
        ex.extract_device(t.data_ptr(), 1, 640, 480, 640, 640 * 480)
        k, d = ex.fetch(0)
        print("torch ptr -> our kernels OK, n=", len(k), flush=True)
    except Exception as e:
        print("torch ptr failed:", e, flush=True)
else:
    import orbslam2_amd as amd
    print("amd devices", amd.device_count(), flush=True)
    ex = amd.ORBextractor(500)
    import torch
    print("torch cuda", torch.cuda.is_available(), flush=True)
