// mi355x_integrator.cpp — the pbrt-side adapter of INTEGRATION.md §2: a pbrt::Integrator whose
// Render() drives the MI355X path through the C-ABI (include/avr.h). It is compiled with pbrt
// (cpu/integrators.h:34-77 is its base class) after the accessor patch of INTEGRATION.md §2a
// (tools/adapter/pbrt_accessors.py applies it to copies of pbrt's headers);
// tests/test_adapter_syntax.py checks with g++ -fsyntax-only that every call below matches
// pbrt's headers and include/avr.h. Registration: one line in Integrator::Create
// (cpu/integrators.cpp:3658-3709), see Mi355xVolPathIntegrator::Create.
//
// Scope: one GridMedium (with its Le or temperature emission) or CloudMedium behind interface
// shapes without material, Distant / UniformInfinite lights, perspective or orthographic
// camera, RGBFilm with a box or Gaussian filter, Independent or ZSobol sampler. The other
// media, image lights, SpectralFilm and multi-GPU contexts follow INTEGRATION.md §2b.
#include <pbrt/cameras.h>
#include <pbrt/cpu/aggregates.h>
#include <pbrt/cpu/integrators.h>
#include <pbrt/cpu/primitive.h>
#include <pbrt/film.h>
#include <pbrt/filters.h>
#include <pbrt/lights.h>
#include <pbrt/media.h>
#include <pbrt/options.h>
#include <pbrt/samplers.h>
#include <pbrt/util/error.h>

#include <memory>
#include <string>
#include <vector>

#include "avr.h"

namespace pbrt {

namespace {

constexpr int kLambdaSamples = 471;   // Lambda_min .. Lambda_max (spectrum.h:36-37)

void CheckAvr(int rc, const char *what) {
    if (rc != AVR_OK)
        ErrorExit("%s failed: %s", what, avr_last_error());
}

void ToRowMajor(const SquareMatrix<4> &m, float out[16]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = m[i][j];
}

void Tabulate(const DenselySampledSpectrum &s, float *out) {
    for (int l = 0; l < kLambdaSamples; ++l) out[l] = s(Lambda_min + l);
}

// The one medium inside the aggregate's interface shapes (graph/util.h:61-91 walks the
// BVHAggregate's GeometricPrimitives the same way)
Medium FindMedium(Primitive aggregate) {
    if (!aggregate.Is<BVHAggregate>())
        ErrorExit("volpath_mi355x: the accelerator must be a BVHAggregate");
    Medium medium = nullptr;
    for (Primitive &p : aggregate.Cast<BVHAggregate>()->GetPrimitives()) {
        if (!p.Is<GeometricPrimitive>())
            ErrorExit("volpath_mi355x: only geometric primitives bound the medium");
        const MediumInterface &mi = p.Cast<GeometricPrimitive>()->GetMediumInterface();
        if (!mi.inside || (medium && medium != mi.inside))
            ErrorExit("volpath_mi355x: exactly one medium inside the interface shapes");
        medium = mi.inside;
    }
    if (!medium)
        ErrorExit("volpath_mi355x: no medium");
    return medium;
}

// DistantLight (lights.h:244-305) and UniformInfiniteLight (lights.h:508-550): type, render-
// space direction towards a distant light (lights.h:287), the emitted spectrum with the
// light's scale folded in (GetLEmit: the same products as scale * Lemit->Sample(lambda))
void UploadLights(avr_context *ctx, const std::vector<Light> &lights, const Bounds3f &sceneBounds) {
    std::vector<int> type;
    std::vector<float> w, L, scale;
    for (Light l : lights) {   // (a copy: GetLEmit / GetRenderFromLight are non-const)
        DenselySampledSpectrum Le;
        if (DistantLight *d = l.CastOrNullptr<DistantLight>()) {
            Vector3f wl = Normalize(d->GetRenderFromLight()(Vector3f(0, 0, 1)));
            type.push_back(0);
            w.insert(w.end(), {wl.x, wl.y, wl.z});
            Le = d->GetLEmit();
        } else if (UniformInfiniteLight *u = l.CastOrNullptr<UniformInfiniteLight>()) {
            type.push_back(1);
            w.insert(w.end(), {0.f, 0.f, 0.f});
            Le = u->GetLEmit();
        } else {
            ErrorExit("volpath_mi355x: %s is not a distant or uniform infinite light", l.ToString());
        }
        scale.push_back(1.f);
        L.resize(L.size() + kLambdaSamples);
        Tabulate(Le, L.data() + L.size() - kLambdaSamples);
    }
    Point3f center;
    Float radius;
    sceneBounds.BoundingSphere(&center, &radius);
    CheckAvr(avr_lights(ctx, (int)type.size(), type.data(), w.data(), L.data(), scale.data(), radius),
             "avr_lights");
}

void UploadMedium(avr_context *ctx, Medium medium) {
    std::vector<float> sa(kLambdaSamples), ss(kLambdaSamples), le(kLambdaSamples);
    float m[16], mi[16], b[6];
    if (GridMedium *gm = medium.CastOrNullptr<GridMedium>()) {        // media.h:265-352
        Tabulate(gm->SigmaASpec(), sa.data());
        Tabulate(gm->SigmaSSpec(), ss.data());
        Tabulate(gm->LeSpec(), le.data());
        const Bounds3f &bb = gm->Bounds();
        const float bounds[6] = {bb.pMin.x, bb.pMin.y, bb.pMin.z, bb.pMax.x, bb.pMax.y, bb.pMax.z};
        ToRowMajor(gm->RenderFromMedium().GetMatrix(), m);
        ToRowMajor(gm->RenderFromMedium().GetInverseMatrix(), mi);
        const SampledGrid<Float> &d = gm->Density(), &ls = gm->LeScaleGrid();
        std::vector<float> dv(d.begin(), d.end()), lv(ls.begin(), ls.end());
        const int mres[3] = {16, 16, 16};                              // media.cpp:229
        const bool emissive = gm->IsEmissive() && !gm->TemperatureGrid();
        CheckAvr(avr_medium_grid(ctx, dv.data(), d.XSize(), d.YSize(), d.ZSize(), bounds, m, mi, sa.data(),
                                 ss.data(), gm->G(), emissive ? le.data() : nullptr, emissive ? lv.data() : nullptr,
                                 ls.XSize(), ls.YSize(), ls.ZSize(), mres),
                 "avr_medium_grid");
        if (const pstd::optional<SampledGrid<Float>> &tg = gm->TemperatureGrid()) {   // media.h:299-316
            std::vector<float> tv(tg->begin(), tg->end());
            CheckAvr(avr_medium_temperature(ctx, tv.data(), gm->TemperatureScale(), gm->TemperatureOffset()),
                     "avr_medium_temperature");
        }
    } else if (CloudMedium *cm = medium.CastOrNullptr<CloudMedium>()) {   // media.h:430-528
        const Bounds3f bb = cm->GetBounds();
        b[0] = bb.pMin.x; b[1] = bb.pMin.y; b[2] = bb.pMin.z; b[3] = bb.pMax.x; b[4] = bb.pMax.y; b[5] = bb.pMax.z;
        ToRowMajor(cm->GetRenderFromMedium().GetMatrix(), m);
        ToRowMajor(cm->GetRenderFromMedium().GetInverseMatrix(), mi);
        Tabulate(cm->SigmaASpec(), sa.data());
        Tabulate(cm->SigmaSSpec(), ss.data());
        CheckAvr(avr_medium_cloud(ctx, b, m, mi, sa.data(), ss.data(), cm->G(), cm->DensityScale(),
                                  cm->Wispiness(), cm->Frequency()),
                 "avr_medium_cloud");
    } else {
        ErrorExit("volpath_mi355x: %s is not a grid or cloud medium", medium.ToString());
    }
}

}  // namespace

// Mi355xVolPathIntegrator: Render() replaces ImageTileIntegrator::Render (integrators.cpp:72-232)
// for the volumetric path; the estimator is VolPathIntegrator::Li (962-1280) on the device.
class Mi355xVolPathIntegrator : public Integrator {
  public:
    Mi355xVolPathIntegrator(int maxDepth, Camera camera, Sampler sampler, Primitive aggregate,
                            std::vector<Light> lights)
        : Integrator(aggregate, lights), maxDepth(maxDepth), camera(camera), samplerPrototype(sampler) {}

    // VolPathIntegrator::Create's parameters (integrators.cpp:1402-1420): maxdepth (default 5)
    static std::unique_ptr<Mi355xVolPathIntegrator> Create(const ParameterDictionary &parameters,
                                                           Camera camera, Sampler sampler,
                                                           Primitive aggregate,
                                                           std::vector<Light> lights, const FileLoc *loc) {
        int maxDepth = parameters.GetOneInt("maxdepth", 5);
        return std::make_unique<Mi355xVolPathIntegrator>(maxDepth, camera, sampler, aggregate, lights);
    }

    void Render() override {
        avr_context *ctx = nullptr;
        CheckAvr(avr_context_create(Options->gpuDevice.value_or(0), 0, &ctx), "avr_context_create");
        UploadMedium(ctx, FindMedium(aggregate));
        UploadLights(ctx, lights, aggregate.Bounds());

        // camera: cameraFromRaster (cameras.h:272) and renderFromCamera at t = 0
        float cfr[16], rfc[16];
        int camType = 1;
        if (PerspectiveCamera *pc = camera.CastOrNullptr<PerspectiveCamera>()) {
            ToRowMajor(pc->CameraFromRaster().GetMatrix(), cfr);
        } else if (OrthographicCamera *oc = camera.CastOrNullptr<OrthographicCamera>()) {
            ToRowMajor(oc->CameraFromRaster().GetMatrix(), cfr);
            camType = 0;
        } else {
            ErrorExit("volpath_mi355x: perspective or orthographic cameras only");
        }
        const CameraTransform &ct = camera.GetCameraTransform();
        ToRowMajor(Inverse(ct.CameraFromRender(0.f)).GetMatrix(), rfc);
        CheckAvr(avr_camera(ctx, camType, cfr, rfc), "avr_camera");

        // film: RGBFilm + its PixelSensor (film.h:95-100, 232-316) and filter
        RGBFilm *film = camera.GetFilm().CastOrNullptr<RGBFilm>();
        if (!film)
            ErrorExit("volpath_mi355x: RGBFilm only");
        const PixelSensor *sensor = film->GetPixelSensor();
        std::vector<float> rgbBar(3 * kLambdaSamples);
        Tabulate(sensor->RBar(), rgbBar.data());
        Tabulate(sensor->GBar(), rgbBar.data() + kLambdaSamples);
        Tabulate(sensor->BBar(), rgbBar.data() + 2 * kLambdaSamples);
        Filter filter = film->GetFilter();
        const Vector2f r = filter.Radius();
        const float radius[2] = {r.x, r.y};
        const Point2i res = film->FullResolution();
        CheckAvr(avr_film(ctx, res.x, res.y, radius, rgbBar.data(), sensor->ImagingRatio(),
                          film->MaxComponentValue()),
                 "avr_film");
        if (GaussianFilter *gf = filter.CastOrNullptr<GaussianFilter>())
            CheckAvr(avr_set_filter(ctx, 1, radius, gf->Sigma()), "avr_set_filter");
        else if (!filter.Is<BoxFilter>())
            ErrorExit("volpath_mi355x: box or gaussian filter only");

        // sampler: IndependentSampler or ZSobolSampler (samplers.h:225-330, 442-476)
        const int spp = samplerPrototype.SamplesPerPixel();
        if (samplerPrototype.Is<ZSobolSampler>())
            CheckAvr(avr_set_sampler(ctx, 1, spp), "avr_set_sampler");
        else if (samplerPrototype.Is<IndependentSampler>())
            CheckAvr(avr_set_sampler(ctx, 0, spp), "avr_set_sampler");
        else
            ErrorExit("volpath_mi355x: independent or zsobol sampler only");

        // render every sample index, then merge the fp64 sums into pbrt's film
        CheckAvr(avr_render(ctx, 0, spp, Options->seed, maxDepth), "avr_render");
        const Bounds2i pb = film->PixelBounds();
        std::vector<double> rgb(3 * (size_t)pb.Area()), w((size_t)pb.Area());
        CheckAvr(avr_film_read(ctx, rgb.data(), w.data()), "avr_film_read");
        size_t i = 0;
        for (Point2i p : pb) {
            film->AddPixelSums(p, &rgb[3 * i], w[i]);
            ++i;
        }
        ImageMetadata metadata;
        camera.InitMetadata(&metadata);
        film->WriteImage(metadata);
        CheckAvr(avr_context_destroy(ctx), "avr_context_destroy");
    }

    std::string ToString() const override { return "[ Mi355xVolPathIntegrator ]"; }

  private:
    int maxDepth;
    Camera camera;
    Sampler samplerPrototype;
};

// The registration line Integrator::Create gains (cpu/integrators.cpp:3678-3700):
//   else if (name == "volpath_mi355x")
//       integrator = Mi355xVolPathIntegrator::Create(parameters, camera, sampler, aggregate, lights, loc);
std::unique_ptr<Integrator> CreateMi355xVolPath(const ParameterDictionary &parameters, Camera camera,
                                                Sampler sampler, Primitive aggregate,
                                                std::vector<Light> lights, const FileLoc *loc) {
    return Mi355xVolPathIntegrator::Create(parameters, camera, sampler, aggregate, lights, loc);
}

}  // namespace pbrt
