// vxpt_offline -- the offline renderer executable over the vxpt C ABI.
//
// Mirrors the reference's mainOffline.cpp (flags :57-133, set-up :140-251, frame loop :273-408,
// canonical gate :423-498) and OfflineBackend::renderFrame / writeAllBatchedFrames
// (OfflineBackend.cpp:46-184).  Host code only: every GPU operation goes through include/vxpt.h.
//
// Same flags and outputs as the reference: saved frames are the 1-indexed {1, 4, 16, 64} written
// as <prefix>_%04d.png with the 0-indexed frame number, the canonical gate compares frame
// totalFrames-1 and writes <prefix>_diff.png.  Additions: --spp (samples per pixel per frame,
// the reference traces 1), --chunks X Y Z (world size, default the reference's 2 1 2), --device,
// --data (the data directory), --perf-report (the run summary file; default <data>/perf/
// performance_report.txt, the reference's data/perf/performance_report.txt), and a per-frame CSV
// <prefix>_frames.csv of the library's timings.
// The scripted voxel-edit sequences (--test-sequence, --test-remove20, --test-remove-circle) follow
// the reference's timing: a click set after frame N is picked at frame N+1 against the world as
// edited so far (VoxelEngine::update, VoxelEngine.cu:906-975) and the geometry changes at frame
// N+2 (OptixRenderer::update rebuilds the chunk's acceleration structure a frame later,
// OptixRenderer.cpp:846-925), the frame whose ReSTIR temporal visibility sees no previous scene.
#include "../../include/vxpt.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <filesystem>
#include <fstream>
#include <future>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>
#include <iomanip>

namespace {

struct Options {
    int width = 3840, height = 2160;
    std::string outputPrefix = "offline_render";
    std::string sceneFile = "data/scene/scene_export.yaml";
    bool testCanonical = false, updateCanonical = false;
    std::string canonicalImagePath = "../../data/canonical/canonical_render.png";
    std::string runComment = "default run";
    int totalFrames = 64;
    std::vector<int> savedFrames = {1, 4, 16, 64};
    int spp = 1;
    int chunks[3] = {2, 1, 2};
    int device = 0;
    std::string dataDir = "data";
    std::string assetsDir;  // root of the instanced meshes' OBJ files (empty: the data directory)
    std::string perfReport;
    bool testSequence = false, removal20 = false, removalCircle = false;
    bool textures = true;
};

void usage(const char *argv0) {
    std::cout << "Offline Voxel Path Tracer (MI355X)\n"
              << "Usage: " << argv0 << " [options]\n"
              << "Options:\n"
              << "  --width <int>          Output width (default: 3840)\n"
              << "  --height <int>         Output height (default: 2160)\n"
              << "  --output <string>      Output filename prefix (default: offline_render)\n"
              << "  --scene <file>         Scene configuration YAML file (camera)\n"
              << "  --test-canonical       Compare output with canonical image\n"
              << "  --update-canonical     Update the canonical reference image\n"
              << "  --canonical-image <p>  Path to canonical image (default: ../../data/canonical/canonical_render.png)\n"
              << "  --comment <text>       Comment for performance report (default: default run)\n"
              << "  --test-sequence        Enable scripted block placement test sequence\n"
              << "  --test-remove20        Enable scripted removal test (20 deletions)\n"
              << "  --test-remove-circle   Enable circular removal test (8 directions, 5 deletions each)\n"
              << "  --frames <int>         Number of frames to render (default: 64, use 1 for single frame)\n"
              << "  --spp <int>            Samples per pixel per frame (default: 1)\n"
              << "  --chunks <x> <y> <z>   World size in 32^3 chunks (default: 2 1 2)\n"
              << "  --device <int>         HIP device (default: 0)\n"
              << "  --data <dir>           Data directory: settings/, assets/, tables/ (default: data)\n"
              << "  --models <dir>         Root of the instanced meshes' OBJ files (<dir>/models/*.obj; default: the data directory)\n"
              << "  --perf-report <file>   Performance report the run summary is appended to\n"
              << "                         (default: <data>/perf/performance_report.txt)\n"
              << "  --no-textures          Untextured materials (textures load from <data>/textures when present)\n"
              << "  --help, -h             Show this help message\n";
}

// returns 1 = run, 0 = exit 0 (help), -1 = exit 2 (bad args)
int parse(int argc, char **argv, Options &o) {
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        // mainOffline.cpp:57-133 reads a flag's value only when one follows (`&& i + 1 < argc`)
        // and skips anything it does not know: a trailing valueless flag and unknown
        // arguments are ignored here too (with a note on stderr), so reference scripts run as-is
        auto next = [&](const char *what) -> const char * {
            if (i + 1 >= argc) {
                std::cerr << "note: " << what << " without a value ignored\n";
                return nullptr;
            }
            return argv[++i];
        };
        const char *v = nullptr;
        if (a == "--width") { if ((v = next("--width"))) { o.width = std::atoi(v); } }
        else if (a == "--height") { if ((v = next("--height"))) { o.height = std::atoi(v); } }
        else if (a == "--output") { if ((v = next("--output"))) { o.outputPrefix = v; } }
        else if (a == "--scene") { if ((v = next("--scene"))) { o.sceneFile = v; } }
        else if (a == "--test-canonical" || a == "--test") o.testCanonical = true;
        else if (a == "--update-canonical") o.updateCanonical = true;
        else if (a == "--canonical-image") { if ((v = next("--canonical-image"))) { o.canonicalImagePath = v; } }
        else if (a == "--comment") { if ((v = next("--comment"))) { o.runComment = v; } }
        else if (a == "--frames") {
            if ((v = next("--frames"))) {
                o.totalFrames = std::atoi(v);
                if (o.totalFrames == 1) o.savedFrames = {1};  // mainOffline.cpp:108-111
            }
        }
        else if (a == "--spp") { if ((v = next("--spp"))) { o.spp = std::atoi(v); } }
        else if (a == "--chunks") {
            for (int k = 0; k < 3; k++) {
                if (!(v = next("--chunks"))) return -1;  // an extension flag: all three values required
                o.chunks[k] = std::atoi(v);
            }
        }
        else if (a == "--device") { if ((v = next("--device"))) { o.device = std::atoi(v); } }
        else if (a == "--data") { if ((v = next("--data"))) { o.dataDir = v; } }
        else if (a == "--models") { if ((v = next("--models"))) { o.assetsDir = v; } }
        else if (a == "--perf-report") { if ((v = next("--perf-report"))) { o.perfReport = v; } }
        else if (a == "--no-textures") o.textures = false;
        else if (a == "--test-sequence") o.testSequence = true;
        else if (a == "--test-remove20") o.removal20 = true;
        else if (a == "--test-remove-circle") o.removalCircle = true;
        else if (a == "--help" || a == "-h") { usage(argv[0]); return 0; }
        else std::cerr << "note: unknown option " << a << " ignored\n";
    }
    if (o.width <= 0 || o.height <= 0) {
        std::cerr << "width and height must be positive\n";
        return -1;
    }
    if (o.totalFrames <= 0 || o.spp <= 0 || o.chunks[0] <= 0 || o.chunks[1] <= 0 || o.chunks[2] <= 0) {
        std::cerr << "frames, spp and chunks must be positive\n";
        return -1;
    }
    if (o.perfReport.empty()) o.perfReport = o.dataDir + "/perf/performance_report.txt";
    return 1;
}

std::string frame_path(const std::string &prefix, int frame0) {
    std::ostringstream s;
    s << prefix << "_" << std::setfill('0') << std::setw(4) << frame0 << ".png";
    return s.str();
}

struct BatchedFrame {
    std::vector<float> rgba;
    std::string path;
};

struct FrameRecord {  // PerformanceTracker's per-frame row, from the library's HIP-event timings
    int frame;
    std::string comment;
    vxpt_timing t;
    double postMs, wallMs;
    float dtMs;
    double updateMs;  // the frame's voxel-engine update on the host (clicks, picks, block edits)
};

// PerformanceTracker's timestamp format (PerformanceTracker.h: "%Y-%m-%d %H:%M:%S.mmm", local time)
std::string timestamp_now() {
    const auto now = std::chrono::system_clock::now();
    const std::time_t tt = std::chrono::system_clock::to_time_t(now);
    const long ms = (long)(std::chrono::duration_cast<std::chrono::milliseconds>(now.time_since_epoch()).count() % 1000);
    std::tm tmv{};
    localtime_r(&tt, &tmv);
    std::ostringstream ss;
    ss << std::put_time(&tmv, "%Y-%m-%d %H:%M:%S") << '.' << std::setfill('0') << std::setw(3) << ms;
    return ss.str();
}

// PerformanceTracker::saveReport (PerformanceTracker.h:98-183): one run-summary line appended to the
// report, the header first when the file is new; columns are per-frame averages in ms.  Here
// PathTrace and Denoiser are the library's HIP-event times (the reference's are CPU launch times),
// ScenePrep is 0 (the sky is built once by vxpt_set_sky, before the loop), RendererUpd the host's
// voxel-engine update.
bool append_run_summary(const std::string &path, const std::string &stamp, int w, int h,
                        const std::vector<FrameRecord> &perf, const std::string &comment) {
    if (perf.empty()) return true;
    const std::filesystem::path fp(path);
    std::error_code ec;
    if (fp.has_parent_path()) std::filesystem::create_directories(fp.parent_path(), ec);
    std::ofstream f(path, std::ios::app);
    if (!f) return false;
    f.seekp(0, std::ios::end);
    if (f.tellp() == 0)
        f << "# Performance Report - Real-time Path Tracing Voxel Renderer (Run Summary)\n"
          << "# Format: Timestamp         | Frames | Resolution | WholeFrame | StdDev | ScenePrep | RendererUpd | "
             "PathTrace | Denoiser | PostProc | Comment\n"
          << "# ==========================================================================================="
             "====================================\n";
    double whole = 0, upd = 0, trace = 0, den = 0, post = 0;
    for (const auto &r : perf) {
        whole += r.wallMs; upd += r.updateMs; trace += r.t.trace_ms; den += r.t.denoise_ms; post += r.postMs;
    }
    const double n = (double)perf.size();
    whole /= n; upd /= n; trace /= n; den /= n; post /= n;
    double var = 0;
    for (const auto &r : perf) var += (r.wallMs - whole) * (r.wallMs - whole);
    const double sd = std::sqrt(var / n);
    f << std::fixed << std::setprecision(2);
    f << std::setw(19) << std::left << stamp << " | ";
    f << std::setw(6) << std::right << perf.size() << " | ";
    f << std::setw(10) << std::left << (std::to_string(w) + "x" + std::to_string(h)) << " | ";
    f << std::setw(10) << std::right << whole << " | ";
    f << std::setw(6) << std::right << sd << " | ";
    f << std::setw(9) << std::right << 0.0 << " | ";
    f << std::setw(11) << std::right << upd << " | ";
    f << std::setw(9) << std::right << trace << " | ";
    f << std::setw(8) << std::right << den << " | ";
    f << std::setw(8) << std::right << post << " | ";
    f << comment << std::endl;
    return (bool)f;
}

void print_diff(const vxpt_image_diff_result &r) {  // ImageDiffResult::print (ImageDiff.cpp)
    std::cout << "=== Image Comparison Results ===\n"
              << "Total pixels: " << r.total_pixels << "\n"
              << "Different pixels: " << r.different_pixels << " (" << std::fixed << std::setprecision(2)
              << r.pixel_difference_ratio * 100.0f << "%)\n"
              << std::setprecision(4) << "RMSE: " << r.rmse << "\n"
              << "SSIM: " << r.ssim << "\n"
              << "Assessment: "
              << (r.is_identical ? "IDENTICAL" : r.is_very_close ? "VERY CLOSE" : r.is_close ? "CLOSE" : "DIFFERENT")
              << "\n";
    std::cout.unsetf(std::ios::floatfield);
}

}  // namespace

int main(int argc, char **argv) {
    Options o;
    const int pr = parse(argc, argv, o);
    if (pr <= 0) return pr == 0 ? 0 : 2;

    std::cout << "=== Offline Voxel Path Tracer ===\n"
              << "Resolution: " << o.width << "x" << o.height << "\n"
              << "Frames to render: " << o.totalFrames << " at " << o.spp << " spp\n"
              << "Output prefix: " << o.outputPrefix << std::endl;

    vxpt_config cfg{};
    cfg.width = o.width;
    cfg.height = o.height;
    cfg.device = o.device;
    cfg.total_bounce_limit = 3;    // RayGen.cu:146
    cfg.diffuse_bounce_limit = 1;  // RayGen.cu:147
    cfg.data_dir = o.dataDir.c_str();
    vxpt_ctx *ctx = nullptr;
    if (vxpt_create(&cfg, &ctx) != VXPT_OK) {
        std::cerr << "Error: vxpt_create failed: " << vxpt_last_error(ctx) << std::endl;
        vxpt_destroy(ctx);
        return 1;
    }
    auto last = std::chrono::steady_clock::now();  // OfflineBackend::init starts m_timer (OfflineBackend.cpp:43)
    auto fail = [&](const char *what) {
        std::cerr << "Error: " << what << ": " << vxpt_last_error(ctx) << std::endl;
        vxpt_destroy(ctx);
        return 1;
    };

    // mainOffline.cpp:140-198: settings, assets, the voxel world
    if (vxpt_load_settings(ctx) != VXPT_OK) return fail("loading settings");
    if (o.textures) {  // TextureManager::initWithMaterialPaths: every material texture found is used
        int nTex = 0;
        if (vxpt_load_textures(ctx, nullptr, &nTex) != VXPT_OK) return fail("loading textures");
        std::cout << "Textures loaded: " << nTex << (nTex ? "" : " (untextured materials)") << std::endl;
    }
    if (vxpt_generate_terrain(ctx, o.chunks[0], o.chunks[1], o.chunks[2], 32.0f, 32.0f * o.chunks[0], 0) != VXPT_OK)
        return fail("generating terrain");
    // VoxelEngine::init (VoxelEngine.cu:809-816): the instanced meshes, their instances in the world and
    // the light table (a full light update); block types whose OBJ file is missing stay empty
    {
        int nModels = 0;
        const int rc = vxpt_load_models(ctx, o.assetsDir.empty() ? nullptr : o.assetsDir.c_str(), &nModels);
        if (rc == VXPT_ERR_IO)  // a data directory without the asset yaml files: no instanced blocks
            std::cout << "Instanced meshes not loaded: " << vxpt_last_error(ctx) << std::endl;
        else if (rc != VXPT_OK)
            return fail("loading the instanced meshes");
        else
            std::cout << "Instanced meshes loaded: " << nModels << std::endl;
    }

    // :200-251: camera from the scene file (defaults when it is absent), history camera = camera
    vxpt_camera cam{};
    const bool haveScene = !o.sceneFile.empty() && std::filesystem::exists(o.sceneFile);
    if (!haveScene && !o.sceneFile.empty())
        std::cout << "Scene file not found: " << o.sceneFile << ", using defaults" << std::endl;
    if (vxpt_load_scene_camera(ctx, haveScene ? o.sceneFile.c_str() : nullptr, &cam) != VXPT_OK)
        return fail("loading the scene camera");
    if (vxpt_set_camera(ctx, &cam, &cam) != VXPT_OK) return fail("setting the camera");
    if (vxpt_set_sky(ctx, 0.25f, 45.0f, 0.0f, 1.0f) != VXPT_OK) return fail("building the sky");
    std::cout << "Camera setup - Position: (" << cam.pos[0] << ", " << cam.pos[1] << ", " << cam.pos[2] << ")\n"
              << "Camera setup - Direction: (" << cam.dir[0] << ", " << cam.dir[1] << ", " << cam.dir[2] << ")\n"
              << "Camera setup - FOV: " << cam.fov_deg << " degrees\n"
              << "Camera movement: DISABLED (static camera)\nStarting rendering..." << std::endl;

    vxpt_denoise_params dp{};
    vxpt_post_params pp{};
    if (vxpt_get_post_params(ctx, &pp) != VXPT_OK) return fail("reading post-process settings");
    if (vxpt_get_denoise_params(ctx, &dp) != VXPT_OK) return fail("reading denoise settings");

    // scripted clicks (mainOffline.cpp:43-50, 166-188, 281-395; VoxelEngine.cu:206-217, 906-945)
    constexpr int kRemovals20 = 20, kDirections = 8, kPerDirection = 5, kCircleRemovals = kDirections * kPerDirection;
    constexpr float kPi = 3.14159265358979323846f, kPiOver180 = kPi / 180.0f, kTwoPi = 2.0f * kPi;
    constexpr float kYawAmp = 12.0f * kPiOver180, kPitchAmp = 6.0f * kPiOver180;
    std::vector<int> clickSequence;  // empty: the default {16, 0, 16} cycle
    if (o.removalCircle) clickSequence.assign(kCircleRemovals, 0);
    else if (o.removal20) clickSequence.assign(kRemovals20, 0);
    size_t clickIndex = 0, defaultIndex = 0;
    bool clickPending = false, editPending = false;
    int edit[4] = {0, 0, 0, 0};
    int removals = 0, circleDone = 0, lastDirection = -1;
    bool circleRestored = false;
    float camInfo[32];
    if (vxpt_get_camera(ctx, 0, camInfo) != VXPT_OK) return fail("reading the camera");
    const float baseYaw = camInfo[30], basePitch = camInfo[31];
    float yaw = baseYaw, pitch = basePitch;

    std::vector<BatchedFrame> batch;
    std::vector<FrameRecord> perf;
    std::string runStamp;
    const size_t frameBytes = (size_t)o.width * o.height * 4 * sizeof(float);

    for (int frame = 0; frame < o.totalFrames; frame++) {  // mainOffline.cpp:273-408
        const int frameNumber = frame + 1;
        const auto t0 = std::chrono::steady_clock::now();
        const float dtMs = std::chrono::duration<float, std::milli>(t0 - last).count();  // Timer::getDeltaTime
        last = t0;
        const bool shouldSave =
            std::find(o.savedFrames.begin(), o.savedFrames.end(), frameNumber) != o.savedFrames.end();
        if (frame == 0) runStamp = timestamp_now();  // PerformanceTracker::beginFrame of the first frame

        // the edit picked last frame reaches the geometry now
        if (editPending) {
            if (vxpt_set_block(ctx, edit[0], edit[1], edit[2], edit[3]) != VXPT_OK) return fail("editing a block");
            editPending = false;
        }
        if (o.removalCircle) {  // mainOffline.cpp:281-305
            if (circleDone < kCircleRemovals) {
                const int dirIndex = circleDone / kPerDirection;
                if (dirIndex != lastDirection) {
                    const float angle = (float)dirIndex * (kTwoPi / (float)kDirections);
                    const float yawOff = (float)(kYawAmp * std::cos(angle)), pitchOff = (float)(kPitchAmp * std::sin(angle));
                    yaw = baseYaw + yawOff;
                    pitch = basePitch + pitchOff;
                    std::cout << "CIRCULAR TEST: Switching to view direction #" << dirIndex + 1 << " (yaw offset "
                              << yawOff << ", pitch offset " << pitchOff << ")" << std::endl;
                    lastDirection = dirIndex;
                }
            } else if (!circleRestored) {
                yaw = baseYaw;
                pitch = basePitch;
                circleRestored = true;
                std::cout << "CIRCULAR TEST: Restored base camera orientation after scripted removals." << std::endl;
            }
            // historyCamera = camera; camera.update() (:278-279, 307)
            if (vxpt_set_camera_angles(ctx, cam.pos, yaw, pitch, cam.fov_deg) != VXPT_OK) return fail("camera");
            std::cout << "CAMERA: frame " << frameNumber << " yaw " << std::hexfloat << yaw << " pitch " << pitch
                      << std::defaultfloat << std::endl;
        }
        if (clickPending) {  // VoxelEngine::update's click, against the world as edited so far
            clickPending = false;
            int blockId;
            if (!clickSequence.empty()) {
                const size_t idx = std::min(clickIndex, clickSequence.size() - 1);
                blockId = clickSequence[idx];
                clickIndex = idx + 1 < clickSequence.size() ? idx + 1 : idx;
            } else {
                static const int defaultSequence[3] = {16, 0, 16};
                blockId = defaultSequence[defaultIndex++ % 3];
            }
            int32_t pk[10];
            if (vxpt_pick_block(ctx, pk) != VXPT_OK) return fail("picking");
            if (blockId == 0 && pk[0]) {
                edit[0] = pk[1]; edit[1] = pk[2]; edit[2] = pk[3]; edit[3] = 0;
                editPending = true;
            } else if (blockId != 0 && pk[5] && pk[0]) {
                edit[0] = pk[6]; edit[1] = pk[7]; edit[2] = pk[8]; edit[3] = blockId;
                editPending = true;
            }
            if (editPending)
                std::cout << "EDIT: frame " << frameNumber << " block " << edit[3] << " at (" << edit[0] << ","
                          << edit[1] << "," << edit[2] << ")" << std::endl;
        }

        const double updateMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (vxpt_render_frame(ctx, &dp, frame, o.spp) != VXPT_OK) return fail("rendering");
        const auto tp = std::chrono::steady_clock::now();
        if (vxpt_postprocess(ctx, &pp, dtMs) != VXPT_OK) return fail("post-processing");
        if (shouldSave) {  // storeFrameInBatch (OfflineBackend.cpp:117-131)
            BatchedFrame b;
            b.rgba.resize((size_t)o.width * o.height * 4);
            if (vxpt_readback(ctx, VXPT_BUF_FRAME, b.rgba.data(), frameBytes) != VXPT_OK)
                return fail("reading the frame");
            b.path = frame_path(o.outputPrefix, frame);
            batch.push_back(std::move(b));
        }
        if (vxpt_sync(ctx) != VXPT_OK) return fail("synchronising");
        const auto t1 = std::chrono::steady_clock::now();
        FrameRecord rec{frameNumber,
                        (shouldSave ? "Saved frame " : "Convergence frame ") + std::to_string(frameNumber) + "/" +
                            std::to_string(o.totalFrames),
                        {}, std::chrono::duration<double, std::milli>(t1 - tp).count(),
                        std::chrono::duration<double, std::milli>(t1 - t0).count(), dtMs, updateMs};
        vxpt_timings(ctx, &rec.t);
        perf.push_back(rec);
        // the clicks the reference scripts after a frame (mainOffline.cpp:346-395)
        if (o.removalCircle) {
            if (circleDone < kCircleRemovals) {
                ++circleDone;
                std::cout << "CIRCULAR TEST: Frame " << frameNumber << " deleting block #" << circleDone << std::endl;
                clickPending = true;
            }
        } else if (o.removal20) {
            if (removals < kRemovals20) {
                ++removals;
                std::cout << "REMOVAL TEST: Frame " << frameNumber << " deleting block #" << removals << std::endl;
                clickPending = true;
            }
        } else if (o.testSequence) {
            if (frameNumber == 2 || frameNumber == 5 || frameNumber == 8) clickPending = true;
        }
        if (shouldSave || frameNumber % 16 == 0)
            std::cout << "Frame " << frameNumber << "/" << o.totalFrames << " completed"
                      << (shouldSave ? " (SAVED)" : "") << std::endl;
    }

    // writeAllBatchedFrames (OfflineBackend.cpp:133-184): PNG encoding in parallel on host threads
    std::cout << "\n=== Rendering Complete - Writing all frames to disk ===" << std::endl;
    std::vector<std::future<int>> writers;
    for (const auto &b : batch)
        writers.push_back(std::async(std::launch::async, [&o, &b] {
            return vxpt_write_png_rgba32f(b.path.c_str(), o.width, o.height, b.rgba.data());
        }));
    int writeErrors = 0;
    for (auto &w : writers) writeErrors += w.get() != VXPT_OK;
    if (writeErrors) {
        std::cerr << "Error: " << writeErrors << " frame(s) failed to write" << std::endl;
        vxpt_destroy(ctx);
        return 1;
    }
    std::cout << "Output files saved with prefix: " << o.outputPrefix << std::endl;

    {  // PerformanceTracker::saveReport: the run summary, and the per-frame rows as a CSV
        const std::string csv = o.outputPrefix + "_frames.csv";
        std::ofstream rep(csv);
        rep << "# " << o.runComment << "\n# " << o.width << "x" << o.height << ", " << o.spp << " spp\n"
            << "frame,trace_ms,denoise_ms,sky_ms,frame_ms,post_ms,wall_ms,dt_ms,comment\n";
        double sumTrace = 0, sumDen = 0, sumWall = 0;
        for (const auto &r : perf) {
            rep << r.frame << "," << r.t.trace_ms << "," << r.t.denoise_ms << "," << r.t.sky_ms << ","
                << r.t.frame_ms << "," << r.postMs << "," << r.wallMs << "," << std::setprecision(9) << r.dtMs
                << std::setprecision(6) << "," << r.comment << "\n";
            sumTrace += r.t.trace_ms;
            sumDen += r.t.denoise_ms;
            sumWall += r.wallMs;
        }
        const double n = (double)perf.size();
        if (!append_run_summary(o.perfReport, runStamp, o.width, o.height, perf, o.runComment))
            std::cerr << "Warning: cannot write the performance report " << o.perfReport << std::endl;
        std::cout << "\n=== Performance Report ===\n"
                  << "avg path tracing " << sumTrace / n << " ms, denoiser " << sumDen / n << " ms, wall "
                  << sumWall / n << " ms per frame\nPerformance data saved to: " << o.perfReport
                  << " (per frame: " << csv << ")" << std::endl;
    }

    int rc = 0;
    if (o.testCanonical || o.updateCanonical) {  // mainOffline.cpp:423-498
        const std::string testImagePath = frame_path(o.outputPrefix, o.totalFrames - 1);
        if (o.updateCanonical) {
            std::cout << "\n=== Updating Canonical Image ===" << std::endl;
            std::error_code ec;
            if (std::filesystem::copy_file(testImagePath, o.canonicalImagePath,
                                           std::filesystem::copy_options::overwrite_existing, ec))
                std::cout << "Canonical image updated: " << o.canonicalImagePath << std::endl;
            else
                std::cerr << "Failed to update canonical image: " << ec.message() << std::endl;
        }
        if (o.testCanonical) {
            std::cout << "\n=== Canonical Image Testing ===" << std::endl;
            if (!std::filesystem::exists(o.canonicalImagePath)) {
                std::cout << "Warning: Canonical image not found at " << o.canonicalImagePath << "\n"
                          << "Use --update-canonical to create it from current render" << std::endl;
            } else if (!std::filesystem::exists(testImagePath)) {
                std::cerr << "Error: Test image not found at " << testImagePath << std::endl;
            } else {
                std::cout << "Comparing: " << testImagePath << " vs " << o.canonicalImagePath << std::endl;
                vxpt_image_diff_result r{};
                if (vxpt_image_diff(testImagePath.c_str(), o.canonicalImagePath.c_str(), &r) != VXPT_OK) {
                    std::cerr << "Error: image comparison failed" << std::endl;
                    rc = 1;
                } else {
                    print_diff(r);
                    const std::string diffPath = o.outputPrefix + "_diff.png";
                    if (vxpt_image_diff_png(testImagePath.c_str(), o.canonicalImagePath.c_str(),
                                            diffPath.c_str()) == VXPT_OK)
                        std::cout << "Difference visualization saved to: " << diffPath << std::endl;
                    else
                        std::cerr << "Failed to generate difference image" << std::endl;
                    if (!r.is_identical && !r.is_very_close) {
                        std::cout << "\nWarning: Significant differences detected from canonical image!\n"
                                  << "This may indicate a regression or intentional change." << std::endl;
                        if (!r.is_close) std::cout << "Consider investigating the differences." << std::endl;
                    } else {
                        std::cout << "\nImage matches canonical reference within acceptable tolerance." << std::endl;
                    }
                }
            }
        }
    }
    vxpt_destroy(ctx);
    return rc;
}
