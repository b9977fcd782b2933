// torch_ext.cpp -- the thin PyTorch-ROCm C++ extension `gaussiansplattingviewer_amd._C`: the
// native entry points the upstream Python package calls, with upstream's signatures, over the C
// ABI of libgsr.so (include/gsr.h).  No kernels here: every launch happens in libgsr.so, on the
// caller's current HIP stream.
//
//   _C.rasterize_gaussians(bg, means3D, colors_precomp, opacities, scales, rotations,
//                          scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tanfovx,
//                          tanfovy, image_height, image_width, sh, sh_degree, campos,
//                          prefiltered, debug)
//       -> (num_rendered, color [3,H,W], radii [P], geomBuffer, binningBuffer, imgBuffer)
//     upstream rasterize_points.cu RasterizeGaussiansCUDA, reached from GaussianRasterizer
//     (renderer_cuda.py:211-224) through _RasterizeGaussians.  The three buffers hold upstream's
//     backward state; the forward-only viewer (renderer_cuda.py:214, torch.no_grad) never reads
//     them, and here they are empty.
//   _C.mark_visible(means3D, viewmatrix, projmatrix) -> bool [P]
//     upstream markVisible (GaussianRasterizer.markVisible).
#include <torch/extension.h>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <mutex>
#include <tuple>
#include <vector>

#include "gsr.h"

namespace {

// One context per device, created on first use; _lib.context(device, 0) renders with the same
// one (context_handle), so both entry paths share a workspace.
std::mutex g_lock;
std::vector<gsr_context *> g_ctx;

gsr_context *context_for(int device) {
    std::lock_guard<std::mutex> lk(g_lock);
    if ((int)g_ctx.size() <= device) g_ctx.resize(device + 1, nullptr);
    if (!g_ctx[device]) {
        c10::hip::HIPGuard guard(device);
        gsr_context *c = nullptr;
        TORCH_CHECK(gsr_create(&c) == GSR_OK, "gsr_create: ", gsr_last_error());
        g_ctx[device] = c;
    }
    return g_ctx[device];
}

// An input as contiguous float32 on means3D's device (copied there if needed, as the Python
// entry does), or nullptr for an absent (empty) optional input (upstream passes
// torch.Tensor([]) for them).  A present input must hold at least `count` values: the kernels
// read the first `count` (upstream reads campos as a vec3 of whatever it is given, and the
// stereo viewer hands a homogeneous 4-vector).
const float *opt_ptr(const torch::Tensor &t, const torch::Device &dev, const char *name,
                     std::vector<torch::Tensor> &keep, int64_t count) {
    if (!t.defined() || t.numel() == 0) return nullptr;
    TORCH_CHECK(t.numel() >= count, name, " holds ", t.numel(), " values, expected ", count);
    torch::Tensor c = t.to(dev, torch::kFloat32).contiguous();
    keep.push_back(c);
    return c.data_ptr<float>();
}

std::tuple<int64_t, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>
rasterize_gaussians(const torch::Tensor &background, const torch::Tensor &means3D,
                    const torch::Tensor &colors, const torch::Tensor &opacity,
                    const torch::Tensor &scales, const torch::Tensor &rotations,
                    double scale_modifier, const torch::Tensor &cov3D_precomp,
                    const torch::Tensor &viewmatrix, const torch::Tensor &projmatrix,
                    double tan_fovx, double tan_fovy, int64_t image_height, int64_t image_width,
                    const torch::Tensor &sh, int64_t degree, const torch::Tensor &campos,
                    bool prefiltered, bool debug) {
    if (means3D.ndimension() != 2 || means3D.size(1) != 3)
        AT_ERROR("means3D must have dimensions (num_points, 3)");
    TORCH_CHECK(means3D.is_cuda(), "means3D must be a device (HIP) tensor");
    const torch::Device dev = means3D.device();
    const int64_t P = means3D.size(0);
    const int64_t H = image_height, W = image_width;
    auto f32 = means3D.options().dtype(torch::kFloat32);
    // upstream zero-fills both; the forward writes every pixel and every radius (P > 0), so
    // only an empty scene needs the fill (two fill kernels fewer per frame)
    torch::Tensor color = P ? torch::empty({3, H, W}, f32) : torch::zeros({3, H, W}, f32);
    torch::Tensor radii = P ? torch::empty({P}, means3D.options().dtype(torch::kInt32))
                            : torch::zeros({P}, means3D.options().dtype(torch::kInt32));
    auto bytes = means3D.options().dtype(torch::kUInt8);
    torch::Tensor geom = torch::empty({0}, bytes), binning = torch::empty({0}, bytes),
                  img = torch::empty({0}, bytes);
    int64_t num_rendered = 0;
    if (P != 0) {
        std::vector<torch::Tensor> keep;
        gsr_gaussians g{};
        g.P = P;
        g.D = (int32_t)degree;
        g.M = !(sh.defined() && sh.numel() != 0) ? 0
              : sh.dim() == 3                ? (int32_t)sh.size(1)
                                             : (int32_t)(sh.numel() / P / 3);
        g.scale_modifier = (float)scale_modifier;
        g.means3D = opt_ptr(means3D, dev, "means3D", keep, 3 * P);
        g.scales = opt_ptr(scales, dev, "scales", keep, 3 * P);
        g.rotations = opt_ptr(rotations, dev, "rotations", keep, 4 * P);
        g.opacities = opt_ptr(opacity, dev, "opacities", keep, P);
        g.shs = opt_ptr(sh, dev, "sh", keep, 3 * (int64_t)g.M * P);
        g.colors_precomp = opt_ptr(colors, dev, "colors_precomp", keep, 3 * P);
        g.cov3D_precomp = opt_ptr(cov3D_precomp, dev, "cov3D_precomp", keep, 6 * P);
        gsr_raster_settings st{};
        st.image_width = (int32_t)W;
        st.image_height = (int32_t)H;
        st.tanfovx = (float)tan_fovx;
        st.tanfovy = (float)tan_fovy;
        st.viewmatrix = opt_ptr(viewmatrix, dev, "viewmatrix", keep, 16);
        st.projmatrix = opt_ptr(projmatrix, dev, "projmatrix", keep, 16);
        st.campos = opt_ptr(campos, dev, "campos", keep, 3);
        st.bg = opt_ptr(background, dev, "bg", keep, 3);
        st.prefiltered = prefiltered ? 1 : 0;
        st.debug = debug ? 1 : 0;
        gsr_outputs out{};
        out.color = color.data_ptr<float>();
        out.radii = radii.data_ptr<int32_t>();
        c10::hip::HIPGuard guard(dev.index());
        gsr_context *ctx = context_for(dev.index());
        hipStream_t s = c10::hip::getCurrentHIPStream(dev.index()).stream();
        int rc;
        {  // the forward waits for K (pinned memory): other Python threads may run meanwhile
            pybind11::gil_scoped_release no_gil;
            rc = gsr_forward(ctx, &g, &st, &out, s);
        }
        TORCH_CHECK(rc == GSR_OK, "gsr_forward failed (", rc, "): ", gsr_last_error());
        num_rendered = out.num_rendered;
    }
    return std::make_tuple(num_rendered, color, radii, geom, binning, img);
}

torch::Tensor mark_visible(const torch::Tensor &means3D, const torch::Tensor &viewmatrix,
                           const torch::Tensor &projmatrix) {
    TORCH_CHECK(means3D.is_cuda(), "means3D must be a device (HIP) tensor");
    const torch::Device dev = means3D.device();
    const int64_t P = means3D.size(0);
    torch::Tensor present = torch::full({P}, false, means3D.options().dtype(torch::kBool));
    if (P != 0) {
        std::vector<torch::Tensor> keep;
        const float *xyz = opt_ptr(means3D, dev, "means3D", keep, 3 * P);
        const float *view = opt_ptr(viewmatrix, dev, "viewmatrix", keep, 16);
        const float *proj = opt_ptr(projmatrix, dev, "projmatrix", keep, 16);
        c10::hip::HIPGuard guard(dev.index());
        gsr_context *ctx = context_for(dev.index());
        hipStream_t s = c10::hip::getCurrentHIPStream(dev.index()).stream();
        const int rc = gsr_mark_visible(ctx, xyz, P, view, proj,
                                        reinterpret_cast<uint8_t *>(present.data_ptr<bool>()), s);
        TORCH_CHECK(rc == GSR_OK, "gsr_mark_visible failed (", rc, "): ", gsr_last_error());
    }
    return present;
}

void release_contexts() {
    std::lock_guard<std::mutex> lk(g_lock);
    for (gsr_context *&c : g_ctx) {
        if (c) gsr_destroy(c);
        c = nullptr;
    }
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "gaussiansplattingviewer_amd native entry points (upstream _C signatures) over libgsr.so";
    m.def("rasterize_gaussians", &rasterize_gaussians,
          "upstream RasterizeGaussiansCUDA: (num_rendered, color, radii, geomBuffer, "
          "binningBuffer, imgBuffer)");
    m.def("mark_visible", &mark_visible, "upstream markVisible: bool[P]");
    m.def("abi_version", []() { return gsr_abi_version(); });
    m.def(
        "context_handle",
        [](int64_t device) { return (uintptr_t)context_for((int)device); },
        "the device's gsr_context (as an address), created on first use");
    m.def("release_contexts", &release_contexts, "destroy every context (process exit)");
}
