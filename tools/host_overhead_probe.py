import os, sys, time, ctypes
sys.path[:0] = ["/root/repo/animating-gaussian-splats_amd", "/root/repo"]
import torch
import splat_scenes as S
from diff_gaussian_rasterization import GaussianRasterizer, _C
import diff_gaussian_rasterization as D
dev = torch.device("cuda", 0)
_C.load_library()
P = 1_000_000
p = S.synthetic_cloud(P, 0.005, sh_degree=3, seed=0, device=dev)
a = S.activated_inputs(p, 3); a.pop("colors_precomp")
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in a.items()}
cam = S.scene_cameras(S.SceneConfig("C3", P, 1920, 1080, 1600.0, 0.005, sh_degree=3, views=S.RIG27), device=dev)[0]
dl = S.upstream_grad(1080, 1920, device=dev)
def T(f, n=50):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n): f()
    dt = (time.perf_counter() - t) / n
    torch.cuda.synchronize()
    return dt * 1e6
img, r, d = GaussianRasterizer(raster_settings=cam)(**leaves)
img.backward(dl, retain_graph=True)
print("autograd backward (retain) us", T(lambda: img.backward(dl, retain_graph=True), 20))
print("CFUNCTYPE thunk us", T(lambda: _C._ALLOC_FN(lambda c, w, n: 0), 200))
print("8 x torch.empty us", T(lambda: [torch.empty((P, 3), device=dev) for _ in range(8)], 200))
print("torch.empty SH us", T(lambda: torch.empty((P, 16, 3), device=dev), 200))
keep = []
print("_camera us", T(lambda: _C._camera(cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy, 1080, 1920, cam.campos, cam.bg, False, []), 200))
print("_gaussians us", T(lambda: _C._gaussians(leaves["means3D"], leaves["shs"], 3, torch.empty(0, device=dev), leaves["opacities"], leaves["scales"], leaves["rotations"], 1.0, torch.empty(0, device=dev), []), 200))
print("_device_guard us", T(lambda: _C._device_guard(dev).__enter__(), 200))
print("_stream_ptr us", T(lambda: _C._stream_ptr(dev), 200))
print("accumulation_target x8 us", T(lambda: [D._accumulation_target(t) for t in leaves.values()], 200))
print("forward (incl K wait) us", T(lambda: GaussianRasterizer(raster_settings=cam)(**leaves), 20))

# split the autograd backward: time spent inside _RasterizeGaussians.backward vs the engine around it
import diff_gaussian_rasterization as D2
orig = D2._RasterizeGaussians.backward
acc = {"inner": 0.0, "n": 0, "c": 0.0}
orig_c = D2._C.rasterize_gaussians_backward
def timed_c(*a, **k):
    t = time.perf_counter(); r = orig_c(*a, **k); acc["c"] += time.perf_counter() - t; return r
D2._C.rasterize_gaussians_backward = timed_c
def timed(ctx, *g):
    t = time.perf_counter(); r = orig(ctx, *g); acc["inner"] += time.perf_counter() - t; acc["n"] += 1; return r
D2._RasterizeGaussians.backward = staticmethod(timed)
img, r, d = GaussianRasterizer(raster_settings=cam)(**leaves)
n = 20
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(n):
    img.backward(dl, retain_graph=True)
tot = (time.perf_counter() - t) / n
torch.cuda.synchronize()
print("backward total us %.1f  inside Function.backward %.1f  inside _C call %.1f" % (tot * 1e6, acc["inner"] / acc["n"] * 1e6, acc["c"] / acc["n"] * 1e6))
# a trivial custom Function on a CUDA tensor: the engine's own overhead
class F(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x * 1
    @staticmethod
    def backward(ctx, g):
        return g
x = torch.zeros(16, device=dev, requires_grad=True)
y = F.apply(x)
gg = torch.ones(16, device=dev)
print("trivial Function backward us", T(lambda: y.backward(gg, retain_graph=True), 200))
