// gsr_bind.cpp -- native argument marshalling for the two per-view calls of the drop-in binding.
//
// diff_gaussian_rasterization/_C.py binds libgsr's C ABI with ctypes.  On a host-bound step (C2: one
// thread submitting 4 views of 100k Gaussians) most of a call's host time was that Python layer, not
// the library (per view: forward 58 us of which 26 us in gsr_forward_*, render half 32 us of which
// 7 us in gsr_backward_render; profiles/r04_c2_host.txt).  This torch extension does the same
// marshalling in C++ for _C._forward, _C.rasterize_gaussians_backward (after its output allocation),
// _C.rasterize_gaussians_backward_render and the per-view part of
// _C.rasterize_gaussians_backward_views: the argument checks
// (same messages), the camera / Gaussian structs, the output and workspace tensors (the caching
// allocator, the same pre-allocated groups as _C._PreAllocator) and the call itself, with the
// interpreter lock released while libgsr runs.  It calls libgsr through the function addresses of the
// library _C.py loaded (set_functions), so there is one library instance in the process (GSR_LIB
// variants included).  It computes nothing of its own: without it _C.py takes its ctypes path.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gsr.h"

namespace py = pybind11;

namespace {

struct Fns {
    decltype(&gsr_forward_info_call) forward_info_call = nullptr;
    decltype(&gsr_forward_async) forward_async = nullptr;
    decltype(&gsr_backward_render) backward_render = nullptr;
    decltype(&gsr_backward_gaussians) backward_gaussians = nullptr;
    decltype(&gsr_backward) backward = nullptr;
    decltype(&gsr_prealloc_alloc) prealloc_alloc = nullptr;
    decltype(&gsr_spec_binning_bytes) spec_binning_bytes = nullptr;
    decltype(&gsr_geom_bytes) geom_bytes = nullptr;
    decltype(&gsr_image_bytes) image_bytes = nullptr;
    decltype(&gsr_scratch_bytes) scratch_bytes = nullptr;
    decltype(&gsr_sums_bytes) sums_bytes = nullptr;
    decltype(&gsr_last_error) last_error = nullptr;
} F;

template <typename T>
void take(const std::map<std::string, int64_t> &a, const char *name, T &dst) {
    auto it = a.find(name);
    if (it == a.end() || !it->second) throw std::runtime_error(std::string("gsr_bind: missing ") + name);
    dst = reinterpret_cast<T>(it->second);
}

void set_functions(const std::map<std::string, int64_t> &a) {
    take(a, "gsr_forward_info_call", F.forward_info_call);
    take(a, "gsr_forward_async", F.forward_async);
    take(a, "gsr_backward_render", F.backward_render);
    take(a, "gsr_backward_gaussians", F.backward_gaussians);
    take(a, "gsr_backward", F.backward);
    take(a, "gsr_prealloc_alloc", F.prealloc_alloc);
    take(a, "gsr_spec_binning_bytes", F.spec_binning_bytes);
    take(a, "gsr_geom_bytes", F.geom_bytes);
    take(a, "gsr_image_bytes", F.image_bytes);
    take(a, "gsr_scratch_bytes", F.scratch_bytes);
    take(a, "gsr_sums_bytes", F.sums_bytes);
    take(a, "gsr_last_error", F.last_error);
}

void check(int rc) {
    if (rc != 0) throw std::runtime_error("libgsr error " + std::to_string(rc) + ": " + F.last_error());
}

bool present(const at::Tensor &t) { return t.defined() && t.numel() > 0; }

const char *torch_name(at::ScalarType t) {  // str(torch.dtype), for the error texts _C.py raises
    switch (t) {
        case at::kDouble: return "torch.float64";
        case at::kHalf: return "torch.float16";
        case at::kBFloat16: return "torch.bfloat16";
        case at::kInt: return "torch.int32";
        case at::kLong: return "torch.int64";
        case at::kShort: return "torch.int16";
        case at::kByte: return "torch.uint8";
        case at::kChar: return "torch.int8";
        case at::kBool: return "torch.bool";
        default: return c10::toString(t);
    }
}

// _C._f32 + _C._ptr: contiguous, on the GPU, float32 -- or NULL for an absent (empty) argument
const float *fptr(const at::Tensor &t, std::vector<at::Tensor> &keep) {
    if (!present(t)) return nullptr;
    if (!t.is_cuda()) throw std::runtime_error("diff_gaussian_rasterization: tensors must be on the GPU (no CPU path)");
    at::Tensor c = t.contiguous();
    if (c.scalar_type() != at::kFloat)
        throw std::runtime_error(std::string("diff_gaussian_rasterization: expected float32, got ") +
                                 torch_name(c.scalar_type()));
    keep.push_back(c);
    return c.data_ptr<float>();
}

// _C._mat16: a 4x4 matrix ((4, 4) or (1, 4, 4), any strides) as fp32 + its (row, col) element strides
const float *mat16(const at::Tensor &m0, int stride[2], std::vector<at::Tensor> &keep) {
    if (m0.numel() != 16) throw std::runtime_error("viewmatrix/projmatrix must hold 16 floats");
    at::Tensor m = m0.scalar_type() == at::kFloat ? m0 : m0.to(at::kFloat);
    const auto sz = m.sizes();
    const bool plain = (m.dim() == 2 && sz[0] == 4 && sz[1] == 4) || (m.dim() == 3 && sz[0] == 1 && sz[1] == 4 && sz[2] == 4);
    if (!plain) m = m.reshape({4, 4});
    stride[0] = (int)m.stride(-2);
    stride[1] = (int)m.stride(-1);
    if (!m.is_cuda()) throw std::runtime_error("diff_gaussian_rasterization: tensors must be on the GPU (no CPU path)");
    keep.push_back(m);
    return m.data_ptr<float>();
}

gsr_camera camera(const at::Tensor &vm, const at::Tensor &pm, double tanfovx, double tanfovy, int H, int W,
                  const at::Tensor &campos, const at::Tensor &bg, bool prefiltered, std::vector<at::Tensor> &keep) {
    gsr_camera c;
    memset(&c, 0, sizeof(c));
    c.image_width = W;
    c.image_height = H;
    c.tan_fovx = (float)tanfovx;
    c.tan_fovy = (float)tanfovy;
    c.viewmatrix = mat16(vm, c.viewmatrix_stride, keep);
    c.projmatrix = mat16(pm, c.projmatrix_stride, keep);
    at::Tensor b = (bg.scalar_type() == at::kFloat && bg.is_contiguous()) ? bg : bg.contiguous().to(at::kFloat);
    c.bg = fptr(b, keep);
    if (present(campos)) {
        at::Tensor cp = (campos.scalar_type() == at::kFloat && campos.dim() == 1) ? campos : campos.reshape({-1}).to(at::kFloat);
        if (!cp.is_cuda()) throw std::runtime_error("diff_gaussian_rasterization: tensors must be on the GPU (no CPU path)");
        keep.push_back(cp);
        c.campos = cp.data_ptr<float>();
        c.campos_stride = (int)cp.stride(0);
    }
    c.prefiltered = prefiltered ? 1 : 0;
    return c;
}

gsr_gaussians gaussians(const at::Tensor &means3D, const at::Tensor &sh, int degree, const at::Tensor &colors,
                        const at::Tensor &opacity, const at::Tensor &scales, const at::Tensor &rotations,
                        double scale_modifier, const at::Tensor &cov3D, int activations, bool prep, int layout,
                        std::vector<at::Tensor> &keep) {
    if (means3D.dim() != 2 || means3D.size(1) != 3) throw std::runtime_error("means3D must have dimensions (num_points, 3)");
    gsr_gaussians g;
    memset(&g, 0, sizeof(g));
    g.P = (int)means3D.size(0);
    g.sh_degree = degree;
    g.sh_coeffs = present(sh) ? (int)sh.size(1) : 0;
    g.scale_modifier = (float)scale_modifier;
    g.means3D = fptr(means3D, keep);
    g.shs = fptr(sh, keep);
    g.colors_precomp = fptr(colors, keep);
    g.opacities = fptr(opacity, keep);
    g.scales = fptr(scales, keep);
    g.rotations = fptr(rotations, keep);
    g.cov3D_precomp = fptr(cov3D, keep);
    g.activations = activations;
    g.prepare_backward = prep ? 1 : 0;
    g.binning_layout = layout;
    return g;
}

// _C._PreAllocator: each group of (buffer kind, bytes) is carved from ONE byte tensor (256-byte
// aligned slices) and handed out by gsr_prealloc_alloc; a request it does not cover falls back to a
// byte tensor made here (no Python)
struct PreAlloc {
    gsr_prealloc pa;
    at::Device dev;
    struct Given { at::Tensor base; int64_t off, bytes; };
    std::map<int, Given> given;
    std::map<int, at::Tensor> fallback;
    explicit PreAlloc(at::Device d) : dev(d) { memset(&pa, 0, sizeof(pa)); }
    void group(std::initializer_list<std::pair<int, size_t>> g, bool on) {
        if (!on) return;
        int64_t total = 0;
        std::vector<std::tuple<int, int64_t, int64_t>> offs;
        for (auto &e : g) {
            offs.emplace_back(e.first, total, (int64_t)e.second);
            total += ((int64_t)e.second + 255) & ~(int64_t)255;
        }
        if (total == 0) return;
        at::Tensor buf = at::empty({total}, at::TensorOptions().dtype(at::kByte).device(dev));
        char *base = (char *)buf.data_ptr();
        for (auto &[w, o, n] : offs)
            if (n > 0) {
                given[w] = Given{buf, o, n};
                pa.ptr[w] = base + o;
                pa.bytes[w] = (size_t)n;
            }
    }
    static void *fallback_fn(void *ctx, int which, size_t bytes) {
        auto *self = static_cast<PreAlloc *>(ctx);
        try {
            at::Tensor t = at::empty({(int64_t)std::max<size_t>(bytes, 1)}, at::TensorOptions().dtype(at::kByte).device(self->dev));
            self->fallback[which] = t;
            return t.data_ptr();
        } catch (...) {
            return nullptr;  // reported through the C ABI as GSR_ERR_ALLOC
        }
    }
    void arm() {
        pa.fallback = &PreAlloc::fallback_fn;
        pa.fallback_ctx = this;
    }
    // (taken: [(which, base, offset, bytes)], fallback: [(which, tensor)]) -- what the call used
    py::tuple result() const {
        py::list taken, fb;
        for (auto &[w, g] : given)
            if ((pa.used >> w) & 1) taken.append(py::make_tuple(w, g.base, g.off, g.bytes));
        for (auto &[w, t] : fallback) fb.append(py::make_tuple(w, t));
        return py::make_tuple(taken, fb);
    }
};

void *raw_stream(at::Device dev) { return (void *)c10::hip::getCurrentHIPStream(dev.index()).stream(); }

// _C._forward: -> (num_rendered, binning_layout, speculated, pending, aux_stream, color, radii, depth,
//                  (taken, fallback))
py::tuple forward(const at::Tensor &bg, const at::Tensor &means3D, const at::Tensor &colors, const at::Tensor &opacity,
                  const at::Tensor &scales, const at::Tensor &rotations, double scale_modifier, const at::Tensor &cov3D,
                  const at::Tensor &viewmatrix, const at::Tensor &projmatrix, double tanfovx, double tanfovy, int H, int W,
                  const at::Tensor &sh, int degree, const at::Tensor &campos, bool prefiltered, int activations,
                  bool prepare_backward, bool speculate, bool nonblocking, bool prealloc) {
    std::vector<at::Tensor> keep;
    gsr_gaussians g = gaussians(means3D, sh, degree, colors, opacity, scales, rotations, scale_modifier, cov3D,
                                activations, prepare_backward, 0, keep);
    gsr_camera cam = camera(viewmatrix, projmatrix, tanfovx, tanfovy, H, W, campos, bg, prefiltered, keep);
    const at::Device dev = means3D.device();
    const int P = g.P;
    auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    at::Tensor color = at::empty({3, H, W}, f32), depth = at::empty({1, H, W}, f32);
    at::Tensor radii = at::empty({P}, at::TensorOptions().dtype(at::kInt).device(dev));
    c10::hip::HIPGuard guard(dev.index());
    const size_t spec = (speculate || nonblocking) && P ? F.spec_binning_bytes(P, W, H, prepare_backward ? 1 : 0) : 0;
    PreAlloc pa(dev);
    pa.group({{GSR_BUF_GEOM, F.geom_bytes(P)}, {GSR_BUF_IMAGE, F.image_bytes(W, H, P)}}, prealloc);
    pa.group({{GSR_BUF_BINNING, spec}}, prealloc);
    pa.arm();
    gsr_forward_info fi;
    memset(&fi, 0, sizeof(fi));
    void *s = raw_stream(dev);
    int rc;
    {
        py::gil_scoped_release nogil;
        rc = nonblocking ? F.forward_async(&cam, &g, F.prealloc_alloc, &pa.pa, color.data_ptr<float>(),
                                           depth.data_ptr<float>(), P ? radii.data_ptr<int>() : nullptr, &fi, s)
                         : F.forward_info_call(&cam, &g, F.prealloc_alloc, &pa.pa, color.data_ptr<float>(),
                                               depth.data_ptr<float>(), P ? radii.data_ptr<int>() : nullptr,
                                               speculate ? 1 : 0, &fi, s);
    }
    check(rc);
    return py::make_tuple(fi.num_rendered, fi.binning_layout, fi.speculated, (unsigned long long)fi.pending,
                          (int64_t)(intptr_t)fi.aux_stream, color, radii, depth, pa.result());
}

// _C.rasterize_gaussians_backward_render: -> (SUMS byte tensor (1 byte when P == 0), (taken, fallback))
py::tuple backward_render(const at::Tensor &bg, const at::Tensor &means3D, const at::Tensor &radii,
                          const at::Tensor &colors, const at::Tensor &scales, const at::Tensor &rotations,
                          double scale_modifier, const at::Tensor &cov3D, const at::Tensor &viewmatrix,
                          const at::Tensor &projmatrix, double tanfovx, double tanfovy, const at::Tensor &dL_dcolor,
                          const at::Tensor &sh, int degree, const at::Tensor &campos, int64_t geom, int R,
                          int64_t binning, int64_t image, int activations, bool prepare_backward, int binning_layout,
                          bool prealloc) {
    std::vector<at::Tensor> keep;
    gsr_gaussians g = gaussians(means3D, sh, degree, colors, at::Tensor(), scales, rotations, scale_modifier, cov3D,
                                activations, prepare_backward, binning_layout, keep);
    const int H = (int)dL_dcolor.size(-2), W = (int)dL_dcolor.size(-1);
    gsr_camera cam = camera(viewmatrix, projmatrix, tanfovx, tanfovy, H, W, campos, bg, false, keep);
    const at::Device dev = means3D.device();
    if (g.P == 0)
        return py::make_tuple(at::empty({1}, at::TensorOptions().dtype(at::kByte).device(dev)),
                              py::make_tuple(py::list(), py::list()));
    at::Tensor dpix = dL_dcolor.contiguous().to(at::kFloat);
    c10::hip::HIPGuard guard(dev.index());
    PreAlloc pa(dev);
    pa.group({{GSR_BUF_SCRATCH, F.scratch_bytes(R >= 0 ? R : binning_layout, W, H)}}, prealloc);
    pa.group({{GSR_BUF_SUMS, F.sums_bytes(g.P)}}, prealloc);
    pa.arm();
    void *s = raw_stream(dev);
    int rc;
    {
        py::gil_scoped_release nogil;
        rc = F.backward_render(&cam, &g, radii.data_ptr<int>(), R, (const void *)geom, (const void *)binning,
                               (const void *)image, dpix.data_ptr<float>(), F.prealloc_alloc, &pa.pa, s);
    }
    check(rc);
    at::Tensor sums;
    if (auto it = pa.fallback.find(GSR_BUF_SUMS); it != pa.fallback.end()) sums = it->second;
    else {
        auto &gv = pa.given.at(GSR_BUF_SUMS);
        sums = gv.base.narrow(0, gv.off, gv.bytes);
    }
    return py::make_tuple(sums, pa.result());
}

void fill_grads(gsr_grads &gr, const std::vector<c10::optional<at::Tensor>> &outs, int acc_bits) {
    memset(&gr, 0, sizeof(gr));
    float **slot[8] = {&gr.dL_dmeans2D, &gr.dL_dcolors, &gr.dL_dopacity, &gr.dL_dmeans3D,
                       &gr.dL_dcov3D, &gr.dL_dsh, &gr.dL_dscales, &gr.dL_drotations};
    for (int k = 0; k < 8 && k < (int)outs.size(); ++k)
        if (outs[k].has_value() && present(*outs[k])) *slot[k] = outs[k]->data_ptr<float>();
    gr.accumulate = acc_bits;
}

// _C.rasterize_gaussians_backward after its output allocation (`outs`: the 8 gradients or None, their
// accumulate bits): the one-call backward of one view
void backward(const at::Tensor &bg, const at::Tensor &means3D, const at::Tensor &radii, const at::Tensor &colors,
              const at::Tensor &scales, const at::Tensor &rotations, double scale_modifier, const at::Tensor &cov3D,
              const at::Tensor &viewmatrix, const at::Tensor &projmatrix, double tanfovx, double tanfovy,
              const at::Tensor &dL_dcolor, const at::Tensor &sh, int degree, const at::Tensor &campos, int64_t geom,
              int R, int64_t binning, int64_t image, int activations, bool prepare_backward, int binning_layout,
              const std::vector<c10::optional<at::Tensor>> &outs, int acc_bits, bool prealloc) {
    std::vector<at::Tensor> keep;
    gsr_gaussians g = gaussians(means3D, sh, degree, colors, at::Tensor(), scales, rotations, scale_modifier, cov3D,
                                activations, prepare_backward, binning_layout, keep);
    const int H = (int)dL_dcolor.size(-2), W = (int)dL_dcolor.size(-1);
    gsr_camera cam = camera(viewmatrix, projmatrix, tanfovx, tanfovy, H, W, campos, bg, false, keep);
    if (g.P == 0) return;
    const at::Device dev = means3D.device();
    at::Tensor dpix = dL_dcolor.contiguous().to(at::kFloat);
    c10::hip::HIPGuard guard(dev.index());
    PreAlloc pa(dev);
    pa.group({{GSR_BUF_SCRATCH, F.scratch_bytes(R, W, H)}}, prealloc);
    pa.arm();
    gsr_grads gr;
    fill_grads(gr, outs, acc_bits);
    void *s = raw_stream(dev);
    int rc;
    {
        py::gil_scoped_release nogil;
        rc = F.backward(&cam, &g, radii.data_ptr<int>(), R, (const void *)geom, (const void *)binning,
                        (const void *)image, dpix.data_ptr<float>(), nullptr, F.prealloc_alloc, &pa.pa, &gr, s);
    }
    check(rc);
}

// Tensor.record_stream(s): the caching allocator keeps t's block from reuse until s's queued work is done
void record(const at::Tensor &t, const c10::hip::HIPStream &s) {
    if (t.defined() && t.is_cuda() && t.storage().data_ptr().get())
        c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), s);
}

std::string dev_str(const at::Device &d) { return d.str(); }

// _C.rasterize_gaussians_backward_views after its output allocation: `views` are the deferred views'
// dicts, `outs` the 8 gradient tensors (or None) with their accumulate bits
void backward_views(const py::list &views, const at::Tensor &means3D, const at::Tensor &colors,
                    const at::Tensor &scales, const at::Tensor &rotations, double scale_modifier, const at::Tensor &cov3D,
                    const at::Tensor &sh, int degree, int activations, const std::vector<c10::optional<at::Tensor>> &outs,
                    int acc_bits) {
    std::vector<at::Tensor> keep;
    gsr_gaussians g = gaussians(means3D, sh, degree, colors, at::Tensor(), scales, rotations, scale_modifier, cov3D,
                                activations, false, 0, keep);
    const int P = g.P;
    const int nv = (int)views.size();
    if (P == 0 || nv == 0) return;
    const at::Device dev = means3D.device();
    c10::hip::HIPGuard guard(dev.index());
    const c10::hip::HIPStream cs = c10::hip::getCurrentHIPStream(dev.index());
    std::vector<gsr_camera> cams(nv);
    std::vector<gsr_view_grad> vg(nv);
    for (int k = 0; k < nv; ++k) {
        const py::dict v = views[k].cast<py::dict>();
        cams[k] = camera(v["viewmatrix"].cast<at::Tensor>(), v["projmatrix"].cast<at::Tensor>(),
                         v["tanfovx"].cast<double>(), v["tanfovy"].cast<double>(), v["image_height"].cast<int>(),
                         v["image_width"].cast<int>(),
                         v["campos"].is_none() ? at::Tensor() : v["campos"].cast<at::Tensor>(),
                         v["bg"].cast<at::Tensor>(), false, keep);
        float *m2p = nullptr;
        if (v.contains("means2D_grad") && !v["means2D_grad"].is_none()) {
            const at::Tensor m2 = v["means2D_grad"].cast<at::Tensor>();
            if (m2.dim() != 2 || m2.size(0) != P || m2.size(1) != 3 || m2.scalar_type() != at::kFloat ||
                !m2.is_contiguous() || m2.device() != dev)
                throw std::runtime_error("views[" + std::to_string(k) + "]['means2D_grad']: expected a contiguous float32 (" +
                                         std::to_string(P) + ", 3) tensor on " + dev_str(dev));
            record(m2, cs);
            m2p = m2.data_ptr<float>();
        }
        const at::Tensor radii = v["radii"].cast<at::Tensor>(), scratch = v["scratch"].cast<at::Tensor>();
        record(radii, cs);
        record(scratch, cs);
        if (v.contains("keep"))
            for (auto h : v["keep"]) record(h.cast<at::Tensor>(), cs);
        const py::object gb = v["geomBuffer"];
        const void *geom;
        if (py::isinstance<py::int_>(gb)) geom = (const void *)gb.cast<int64_t>();
        else {
            const at::Tensor gt = gb.cast<at::Tensor>();
            record(gt, cs);
            geom = gt.data_ptr();
        }
        vg[k].cam = &cams[k];
        vg[k].radii = radii.data_ptr<int>();
        vg[k].geom = geom;
        vg[k].scratch = scratch.data_ptr();
        vg[k].num_rendered = v["num_rendered"].cast<int>();
        vg[k].dL_dmeans2D = m2p;
        vg[k].accumulate_means2D = (v.contains("accumulate_means2D") && v["accumulate_means2D"].cast<bool>()) ? 1 : 0;
    }
    gsr_grads gr;
    fill_grads(gr, outs, acc_bits);
    void *s = (void *)cs.stream();
    int rc;
    {
        py::gil_scoped_release nogil;
        rc = F.backward_gaussians(nv, vg.data(), &g, &gr, s);
    }
    check(rc);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "native argument marshalling for diff_gaussian_rasterization._C (libgsr's C ABI)";
    m.def("set_functions", &set_functions);
    // the include/gsr.h ABI this build's structs follow: _C.py falls back to ctypes when it differs
    // from the loaded library's gsr_abi_version() (a stale build would pass wrongly sized structs)
    m.def("abi_version", []() { return (int)GSR_ABI_VERSION; });
    m.def("forward", &forward);
    m.def("backward_render", &backward_render);
    m.def("backward_views", &backward_views);
    m.def("backward", &backward);
}
