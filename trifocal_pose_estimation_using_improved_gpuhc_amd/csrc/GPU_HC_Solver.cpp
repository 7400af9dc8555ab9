// GPU_HC_Solver.cpp -- C++ host driver over the C-ABI (include/hc_trifocal.h).
//
// Follows magmaHC/GPU_HC_Solver.cpp member for member (line citations below);
// MAGMA queues become one HIP stream per device, magma_c{set,get}matrix become
// hipMemcpyAsync, the L2 persisting window is not needed (the compacted index
// tables live in LDS), and every kernel launch goes through the C-ABI.
#include "../../include/GPU_HC_Solver.hpp"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

#include "../../include/hc_host.h"

#define HC_HIP_CHECK(call)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) +      \
                                     " at " + __FILE__ + ":" + std::to_string(__LINE__));    \
    } while (0)

namespace {
constexpr int NV = 30, NPP = 34, NT = 312;

std::string trim(const std::string &s) {
    const auto b = s.find_first_not_of(" \t\r\n");
    if (b == std::string::npos) return "";
    const auto e = s.find_last_not_of(" \t\r\n");
    return s.substr(b, e - b + 1);
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

// ------------------------------------------------------------------ settings
HC_Settings HC_Settings::LoadFile(const std::string &path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open settings file " + path);
    HC_Settings s;
    std::string line;
    while (std::getline(f, line)) {
        const auto h = line.find('#');
        if (h != std::string::npos) line = line.substr(0, h);
        line = trim(line);
        if (line.empty() || line[0] == '%') continue;
        const auto c = line.find(':');
        if (c == std::string::npos) continue;
        s.kv_[trim(line.substr(0, c))] = trim(line.substr(c + 1));
    }
    return s;
}
std::string HC_Settings::str(const std::string &k) const {
    auto it = kv_.find(k);
    if (it == kv_.end()) throw std::runtime_error("missing settings key " + k);
    return it->second;
}
int HC_Settings::i(const std::string &k, int dflt) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? dflt : std::stoi(it->second);
}
bool HC_Settings::b(const std::string &k, bool dflt) const {
    auto it = kv_.find(k);
    if (it == kv_.end()) return dflt;
    return it->second == "true" || it->second == "True" || it->second == "1";
}

// ------------------------------------------------------------------ per-GPU state
struct GPU_HC_Solver::PerGPU {
    int dev = 0, g = 0, N = 0;   // HIP device, logical GPU index (== dev unless Share_Devices)
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hcComplex *d_Start_Sols = nullptr, *d_Track = nullptr, *d_Start_Params = nullptr;
    hcComplex *d_Target_Params = nullptr, *d_diffParams = nullptr;
    int32_t *d_unified_index = nullptr;
    uint8_t *d_conv = nullptr, *d_inf = nullptr;
    hcPathStats *d_stats = nullptr;
    void *d_ws = nullptr;
    size_t ws_bytes = 0;
    // abort mode
    float *d_edgels = nullptr, *d_K = nullptr;
    uint8_t *d_found = nullptr;
    int32_t *d_batch_index = nullptr;
    // pose recovery / maximal support (hc_pose.h), every run
    int32_t *d_inliers = nullptr;
    hcPoseSelection *d_sel = nullptr;
    hcPoseSelection h_sel{};
    int edgel_capacity = 0;
    std::vector<hcComplex> h_track;
    std::vector<uint8_t> h_conv, h_inf;
    std::vector<hcPathStats> h_stats;
    std::vector<int32_t> h_batch_index;
    uint8_t h_found = 0;
};

GPU_HC_Solver::GPU_HC_Solver(const HC_Settings &S, const std::string &root_dir) {
    // GPU_HC_Solver.cpp:44-66
    HC_problem = S.str("problem_name");
    HC_print_problem_name = S.has("problem_print_out_name") ? S.str("problem_print_out_name") : HC_problem;
    GPUHC_Max_Steps = S.i("GPUHC_Max_Steps", 80);
    GPUHC_Max_Correction_Steps = S.i("GPUHC_Max_Correction_Steps", 3);
    GPUHC_delta_t_incremental_steps = S.i("GPUHC_Num_Of_Steps_to_Increase_Delta_t", 4);
    Num_Of_Vars = S.i("Num_Of_Vars", 30);
    Num_Of_Params = S.i("Num_Of_Params", 33);
    Num_Of_Tracks = S.i("Num_Of_Tracks", 312);
    Abort_RANSAC_by_Good_Sol = S.b("Abort_RANSAC_by_Good_Sol", false);
    Abort_Inflight_Stop = S.b("Abort_Inflight_Stop", false);
    Abort_Across_GPUs = S.b("Abort_Across_GPUs", false);
    RANSAC_Dataset_Name = S.has("RANSAC_Dataset") ? S.str("RANSAC_Dataset") : "Synthetic";
    Num_Of_GPUs = S.i("Num_Of_GPUs", 1);
    Num_Of_RANSAC_Iterations = S.i("Num_Of_RANSAC_Iterations", 100);
    Pose_Flags = S.b("Pose_Selection_Reference_Quirks", false) ? HC_POSE_REFERENCE_QUIRKS : 0;
    if (HC_problem != "trifocal_2op1p_30x30" || Num_Of_Vars != NV || Num_Of_Params != NPP - 1 || Num_Of_Tracks != NT)
        throw std::runtime_error("this build implements trifocal_2op1p_30x30 (30 vars, 33 params, 312 tracks) only");
    int device_count = 0;
    HC_HIP_CHECK(hipGetDeviceCount(&device_count));
    // check_multiGPUs (GPU_HC_Solver.hpp:175-193), reported as exceptions instead of exit(1)
    if (Num_Of_GPUs < 1 || Num_Of_GPUs > MAX_NUM_OF_GPUS)
        throw std::runtime_error("Num_Of_GPUs must be in [1, " + std::to_string(MAX_NUM_OF_GPUS) + "]");
    // Share_Devices (not in the reference): more logical GPUs than devices, logical
    // GPU g on device g % device_count with its own stream and buffers -- the
    // multi-GPU split, launch loop and result stacking on a single-GPU machine
    const bool share = S.b("Share_Devices", false);
    if (Num_Of_GPUs > device_count && !share) throw std::runtime_error("Not enough GPUs");
    if (device_count < 1) throw std::runtime_error("no GPU");
    hc_split_samples(Num_Of_RANSAC_Iterations, Num_Of_GPUs, sub_RANSAC_iters);   // :85-88
    for (int g = 0; g < Num_Of_GPUs; g++) {
        printf("GPU %2d computes %2d RANSAC iterations\n", g, sub_RANSAC_iters[g]);
        auto *p = new PerGPU();
        p->g = g;
        p->dev = g % device_count;
        p->N = sub_RANSAC_iters[g];
        HC_HIP_CHECK(hipSetDevice(p->dev));
        HC_HIP_CHECK(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
        HC_HIP_CHECK(hipEventCreate(&p->ev0));
        HC_HIP_CHECK(hipEventCreate(&p->ev1));
        gpus_.push_back(p);
    }
    // reference layout <root>/problems/<p>, <root>/RANSAC_Data/<p>/<dataset> (:128-130);
    // this repository keeps them under <root>/data/
    std::string root = root_dir;
    if (!root.empty() && root.back() != '/') root += '/';
    std::ifstream probe(root + "problems/" + HC_problem + "/start_sols.txt");
    const std::string base = probe ? root : root + "data/";
    Problem_File_Path = base + "problems/" + HC_problem;
    RANSAC_Data_File_Path = base + "RANSAC_Data/" + HC_problem + "/" + RANSAC_Dataset_Name;
    Write_Files_Path = root + "Output_Write_Files/";
}

void GPU_HC_Solver::Allocate_Arrays() {
    // GPU_HC_Solver.cpp:137-184
    h_Start_Sols.assign((size_t)NT * (NV + 1) * 2, 0.0f);
    h_Start_Params.assign(NPP * 2, 0.0f);
    h_unified_dHdx_dHdt_Index.assign(HC_UNIFIED_INDEX_SIZE, 0);
    h_Target_Params.assign((size_t)Num_Of_RANSAC_Iterations * NPP * 2, 0.0f);
    h_diffParams.assign((size_t)Num_Of_RANSAC_Iterations * NPP * 2, 0.0f);
    h_picked.assign((size_t)Num_Of_RANSAC_Iterations * 3, 0);
    for (PerGPU *p : gpus_) {
        // room for time slicing of this GPU's tracking launch (hc_trifocal_workspace_size_for_steps)
        const size_t wsb = hc_trifocal_workspace_size_for_steps(p->N, GPUHC_Max_Steps);
        HC_HIP_CHECK(hipSetDevice(p->dev));
        const size_t n = (size_t)NT * p->N;
        HC_HIP_CHECK(hipMalloc(&p->d_Start_Sols, (size_t)NT * (NV + 1) * sizeof(hcComplex)));
        HC_HIP_CHECK(hipMalloc(&p->d_Track, std::max<size_t>(1, n) * (NV + 1) * sizeof(hcComplex)));
        HC_HIP_CHECK(hipMalloc(&p->d_Start_Params, NPP * sizeof(hcComplex)));
        HC_HIP_CHECK(hipMalloc(&p->d_Target_Params, std::max(1, p->N) * NPP * sizeof(hcComplex)));
        HC_HIP_CHECK(hipMalloc(&p->d_diffParams, std::max(1, p->N) * NPP * sizeof(hcComplex)));
        HC_HIP_CHECK(hipMalloc(&p->d_unified_index, HC_UNIFIED_INDEX_SIZE * sizeof(int32_t)));
        HC_HIP_CHECK(hipMalloc(&p->d_conv, std::max<size_t>(1, n)));
        HC_HIP_CHECK(hipMalloc(&p->d_inf, std::max<size_t>(1, n)));
        HC_HIP_CHECK(hipMalloc(&p->d_stats, std::max<size_t>(1, n) * sizeof(hcPathStats)));
        HC_HIP_CHECK(hipMalloc(&p->d_ws, wsb));
        HC_HIP_CHECK(hipMalloc(&p->d_inliers, std::max<size_t>(1, n) * 2 * sizeof(int32_t)));
        HC_HIP_CHECK(hipMalloc(&p->d_sel, sizeof(hcPoseSelection)));
        p->ws_bytes = wsb;
        p->h_track.resize(n * (NV + 1));
        p->h_conv.resize(n);
        p->h_inf.resize(n);
        p->h_stats.resize(n);
    }
}

bool GPU_HC_Solver::Read_Problem_Data() {
    // GPU_HC_Solver.cpp:186-222 through Data_Reader semantics (hc_host.h)
    const std::string d = Problem_File_Path;
    if (hc_read_start_params((d + "/start_params.txt").c_str(), h_Start_Params.data()) != NPP - 1) {
        printf("[DATA LOAD ERROR] Start Parameters not loaded successfully!\n");
        return false;
    }
    if (hc_read_start_sols((d + "/start_sols.txt").c_str(), h_Start_Sols.data()) != NT * NV) {
        printf("[DATA LOAD ERROR] Start Solutions not loaded successfully!\n");
        return false;
    }
    if (hc_read_int_table((d + "/dHdx_indx.txt").c_str(), h_unified_dHdx_dHdt_Index.data(), 36000) != 36000) {
        printf("[DATA LOAD ERROR] dH/dx Evaluation Indices not loaded successfully!\n");
        return false;
    }
    if (hc_read_int_table((d + "/dHdt_indx.txt").c_str(), h_unified_dHdx_dHdt_Index.data() + 36000, 2880) != 2880) {
        printf("[DATA LOAD ERROR] dH/dt Evaluation Indices not loaded successfully!\n");
        return false;
    }
    return true;
}

bool GPU_HC_Solver::Read_RANSAC_Data(int tp_index) {
    // GPU_HC_Solver.cpp:224-250, Data_Reader.cpp:191-338
    char idx[16];
    snprintf(idx, sizeof(idx), "%03d", tp_index);
    const std::string d = RANSAC_Data_File_Path;
    const std::string f = d + "/Triplet_Edgels/Triplet_Edgels_" + idx + ".txt";
    Num_Of_Triplet_Edgels = hc_count_triplet_edgels(f.c_str());
    if (Num_Of_Triplet_Edgels == 0) {
        printf("[ERROR] File %s not found!\n", f.c_str());
        return false;
    }
    h_Triplet_Edge_Locations.assign((size_t)Num_Of_Triplet_Edgels * 6, 0.0f);
    h_Triplet_Edge_Tangents.assign((size_t)Num_Of_Triplet_Edgels * 6, 0.0f);
    if (hc_read_float_table((d + "/GT_Poses21/GT_Poses21_" + idx + ".txt").c_str(), h_Camera_Pose21, 12) < 0 ||
        hc_read_float_table((d + "/GT_Poses31/GT_Poses31_" + idx + ".txt").c_str(), h_Camera_Pose31, 12) < 0) {
        printf("[DATA LOAD ERROR] Camera Extrinsic Matrices not loaded successfully!\n");
        return false;
    }
    if (hc_read_float_table((d + "/Intrinsic_Matrix.txt").c_str(), h_Camera_Intrinsic_Matrix, 9) != 9) {
        printf("[DATA LOAD ERROR] Camera Intrinsic Matrices not loaded successfully!\n");
        return false;
    }
    hc_read_triplet_edgels(f.c_str(), h_Triplet_Edge_Locations.data(), h_Triplet_Edge_Tangents.data(),
                           Num_Of_Triplet_Edgels);
    return true;
}

void GPU_HC_Solver::Prepare_Target_Params(unsigned rand_seed_) {
    // GPU_HC_Solver.cpp:252-306 (srand(seed), gpu-major / sample-minor draws)
    hc_prepare_target_params(rand_seed_, Num_Of_GPUs, sub_RANSAC_iters, h_Triplet_Edge_Locations.data(),
                             h_Triplet_Edge_Tangents.data(), Num_Of_Triplet_Edgels, h_Start_Params.data(),
                             h_Target_Params.data(), h_diffParams.data(), h_picked.data());
}

void GPU_HC_Solver::Set_RANSAC_Abort_Arrays() {
    // GPU_HC_Solver.cpp:308-333
    if (!Abort_RANSAC_by_Good_Sol) return;
    for (PerGPU *p : gpus_) {
        HC_HIP_CHECK(hipSetDevice(p->dev));
        const size_t n = (size_t)NT * p->N;
        HC_HIP_CHECK(hipMalloc(&p->d_found, 1));
        HC_HIP_CHECK(hipMalloc(&p->d_batch_index, std::max<size_t>(1, n) * sizeof(int32_t)));
        p->h_batch_index.assign(n, -1);
        p->h_found = 0;
    }
    // Abort_Across_GPUs (not in the reference, which keeps one flag per GPU,
    // GPU_HC_Solver.cpp:308-333): a 4-byte flag on the first GPU's device that
    // every GPU's launch sets on a find and polls before each path
    // (hcAbortArgs::peer_found, system-scope atomics over xGMI).  Uncached
    // device memory: coherent across devices while the kernels run (plain
    // hipMalloc memory is coherent only at synchronisation points)
    if (Abort_Across_GPUs && !gpus_.empty() && !d_peer_found) {
        const int dev0 = gpus_[0]->dev;
        for (PerGPU *p : gpus_) {
            if (p->dev == dev0) continue;
            HC_HIP_CHECK(hipSetDevice(p->dev));
            const hipError_t e = hipDeviceEnablePeerAccess(dev0, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HC_HIP_CHECK(e);
            (void)hipGetLastError();
        }
        HC_HIP_CHECK(hipSetDevice(dev0));
        // the same order as hc_shared_flag_create: uncached, fine-grained, then
        // plain memory as the last resort (said once on stderr)
        static const char *const kind_name[3] = {"uncached", "fine-grained", "coarse-grained (hipMalloc)"};
        hipError_t e = hipErrorOutOfMemory;
        for (int k = 0; k < 3 && !d_peer_found; k++) {
            e = k == 0 ? hipExtMallocWithFlags((void **)&d_peer_found, 256, hipDeviceMallocUncached)
              : k == 1 ? hipExtMallocWithFlags((void **)&d_peer_found, 256, hipDeviceMallocFinegrained)
                       : hipMalloc((void **)&d_peer_found, 256);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                d_peer_found = nullptr;
                continue;
            }
            peer_flag_kind_ = kind_name[k];
            if (k > 0)
                fprintf(stderr, "[GPU_HC_Solver] Abort_Across_GPUs: the found flag is in %s memory\n", kind_name[k]);
        }
        HC_HIP_CHECK(e);
        HC_HIP_CHECK(hipMemset(d_peer_found, 0, 256));
    }
}

void GPU_HC_Solver::Data_Transfer_From_Host_To_Device() {
    // GPU_HC_Solver.cpp:335-362; tracks start at the start solutions
    // (Feed_Start_Sols_for_Intermediate_Homotopy, Data_Reader.cpp:62-84)
    int offset = 0;
    for (PerGPU *p : gpus_) {
        HC_HIP_CHECK(hipSetDevice(p->dev));
        const double t0 = now_s();
        const size_t sol_bytes = (size_t)NT * (NV + 1) * sizeof(hcComplex);
        HC_HIP_CHECK(hipMemcpyAsync(p->d_Start_Sols, h_Start_Sols.data(), sol_bytes, hipMemcpyHostToDevice, p->stream));
        for (int k = 0; k < p->N; k++)
            HC_HIP_CHECK(hipMemcpyAsync((char *)p->d_Track + k * sol_bytes, p->d_Start_Sols, sol_bytes,
                                        hipMemcpyDeviceToDevice, p->stream));
        HC_HIP_CHECK(hipMemcpyAsync(p->d_Start_Params, h_Start_Params.data(), NPP * sizeof(hcComplex),
                                    hipMemcpyHostToDevice, p->stream));
        if (p->N > 0) {
            HC_HIP_CHECK(hipMemcpyAsync(p->d_Target_Params, h_Target_Params.data() + (size_t)offset * NPP * 2,
                                        (size_t)p->N * NPP * sizeof(hcComplex), hipMemcpyHostToDevice, p->stream));
            HC_HIP_CHECK(hipMemcpyAsync(p->d_diffParams, h_diffParams.data() + (size_t)offset * NPP * 2,
                                        (size_t)p->N * NPP * sizeof(hcComplex), hipMemcpyHostToDevice, p->stream));
        }
        HC_HIP_CHECK(hipMemcpyAsync(p->d_unified_index, h_unified_dHdx_dHdt_Index.data(),
                                    HC_UNIFIED_INDEX_SIZE * sizeof(int32_t), hipMemcpyHostToDevice, p->stream));
        // triplet edgels + K: abort-mode scoring and the pose recovery of every run
        if (p->d_edgels && p->edgel_capacity < Num_Of_Triplet_Edgels) {
            HC_HIP_CHECK(hipFree(p->d_edgels));
            p->d_edgels = nullptr;
        }
        if (!p->d_edgels) {
            HC_HIP_CHECK(hipMalloc(&p->d_edgels, (size_t)std::max(1, Num_Of_Triplet_Edgels) * 6 * sizeof(float)));
            p->edgel_capacity = Num_Of_Triplet_Edgels;
        }
        if (!p->d_K) HC_HIP_CHECK(hipMalloc(&p->d_K, 9 * sizeof(float)));
        HC_HIP_CHECK(hipMemcpyAsync(p->d_edgels, h_Triplet_Edge_Locations.data(),
                                    (size_t)Num_Of_Triplet_Edgels * 6 * sizeof(float), hipMemcpyHostToDevice,
                                    p->stream));
        HC_HIP_CHECK(hipMemcpyAsync(p->d_K, h_Camera_Intrinsic_Matrix, 9 * sizeof(float), hipMemcpyHostToDevice,
                                    p->stream));
        if (Abort_RANSAC_by_Good_Sol) {
            HC_HIP_CHECK(hipMemcpyAsync(p->d_batch_index, p->h_batch_index.data(),
                                        p->h_batch_index.size() * sizeof(int32_t), hipMemcpyHostToDevice, p->stream));
            HC_HIP_CHECK(hipMemsetAsync(p->d_found, 0, 1, p->stream));
            if (d_peer_found && p == gpus_.front())
                HC_HIP_CHECK(hipMemsetAsync(d_peer_found, 0, sizeof(uint32_t), p->stream));
        }
        HC_HIP_CHECK(hipStreamSynchronize(p->stream));
        transfer_h2d_time[p->g] = now_s() - t0;
        offset += p->N;
    }
}

void GPU_HC_Solver::Set_CUDA_Stream_Attributes() {
    // GPU_HC_Solver.cpp:364-378 sets an L2 access-policy window over the index
    // table on Ampere+.  Not needed on CDNA: the kernel compacts the table into LDS.
}

void GPU_HC_Solver::Solve_by_GPU_HC() {
    // GPU_HC_Solver.cpp:380-566
    std::cout << "GPU computing ..." << std::endl << std::endl;
    multi_GPUs_time = now_s();                                                  // :384
    for (PerGPU *p : gpus_) {                                                   // :390-436
        HC_HIP_CHECK(hipSetDevice(p->dev));
        hcTrackArgs a;
        std::memset(&a, 0, sizeof(a));
        a.sub_ransac_iters = p->N;
        a.settings.max_steps = GPUHC_Max_Steps;
        a.settings.max_corrections = GPUHC_Max_Correction_Steps;
        a.settings.delta_t_inc_steps = GPUHC_delta_t_incremental_steps;
        a.start_sols = p->d_Start_Sols;
        a.tracks = p->d_Track;
        a.start_params = p->d_Start_Params;
        a.target_params = p->d_Target_Params;
        a.diff_params = p->d_diffParams;
        a.unified_index = p->d_unified_index;
        a.converge = p->d_conv;
        a.infinity = p->d_inf;
        a.stats = p->d_stats;
        HC_HIP_CHECK(hipEventRecord(p->ev0, p->stream));
        hcStatus st;
        if (Abort_RANSAC_by_Good_Sol) {
            hcAbortArgs ab;
            std::memset(&ab, 0, sizeof(ab));
            ab.num_triplet_edgels = Num_Of_Triplet_Edgels;
            ab.triplet_edge_locations = p->d_edgels;
            ab.intrinsic_matrix = p->d_K;
            ab.found_trifocal_sols = p->d_found;
            ab.trifocal_sols_batch_index = p->d_batch_index;
            ab.inflight_stop = Abort_Inflight_Stop ? 1 : 0;
            ab.peer_found = d_peer_found;
            st = hc_trifocal_2op1p_30x30_track_abort(&a, &ab, p->d_ws, p->ws_bytes, (hcStream)p->stream);
        } else {
            st = hc_trifocal_2op1p_30x30_track(&a, p->d_ws, p->ws_bytes, (hcStream)p->stream);
        }
        if (st != HC_SUCCESS)
            throw std::runtime_error(std::string("GPU-HC launch failed: status ") + std::to_string((int)st) + " (" +
                                     hc_last_error_string() + ")");
        HC_HIP_CHECK(hipEventRecord(p->ev1, p->stream));
    }
    for (PerGPU *p : gpus_) {                                                   // :440-444
        HC_HIP_CHECK(hipSetDevice(p->dev));
        HC_HIP_CHECK(hipStreamSynchronize(p->stream));
    }
    multi_GPUs_time = now_s() - multi_GPUs_time;                                // :446
    for (PerGPU *p : gpus_) {
        HC_HIP_CHECK(hipSetDevice(p->dev));
        const hcStatus st = hc_trifocal_workspace_status(p->d_ws);
        if (st != HC_SUCCESS)
            throw std::runtime_error(std::string("GPU-HC tracking failed on device ") + std::to_string(p->dev) +
                                     ": status " + std::to_string((int)st));
    }

    // Transform_GPUHC_Sols_to_Trifocal_Relative_Pose + get_Solution_with_Maximal_Support
    // (:526-527), on the device before the copies back, outside the tracking timer
    // like the reference's host evaluation
    const double tp = now_s();
    for (PerGPU *p : gpus_) {
        HC_HIP_CHECK(hipSetDevice(p->dev));
        const hcStatus st = hc_trifocal_pose_support(NT * p->N, p->d_Track, p->d_conv, Num_Of_Triplet_Edgels,
                                                     p->d_edgels, p->d_K, Pose_Flags, p->d_inliers, p->d_sel,
                                                     (hcStream)p->stream);
        if (st != HC_SUCCESS)
            throw std::runtime_error(std::string("pose support launch failed: status ") + std::to_string((int)st) +
                                     " (" + hc_last_error_string() + ")");
        HC_HIP_CHECK(hipMemcpyAsync(&p->h_sel, p->d_sel, sizeof(hcPoseSelection), hipMemcpyDeviceToHost, p->stream));
    }
    for (PerGPU *p : gpus_) {
        HC_HIP_CHECK(hipSetDevice(p->dev));
        HC_HIP_CHECK(hipStreamSynchronize(p->stream));
    }
    pose_time = now_s() - tp;

    h_GPU_HC_Track_Sols_Stack.clear();
    h_is_GPU_HC_Sol_Converge_Stack.clear();
    h_is_GPU_HC_Sol_Infinity_Stack.clear();
    h_Path_Stats_Stack.clear();
    h_Batch_Index_Stack.clear();
    h_Found_Stack.clear();
    for (PerGPU *p : gpus_) {                                                   // :449-460, :494-506
        HC_HIP_CHECK(hipSetDevice(p->dev));
        float ms = 0.0f;
        HC_HIP_CHECK(hipEventElapsedTime(&ms, p->ev0, p->ev1));
        gpu_time[p->g] = ms / 1e3;
        const double t0 = now_s();
        const size_t n = (size_t)NT * p->N;
        if (n) {
            HC_HIP_CHECK(hipMemcpy(p->h_track.data(), p->d_Track, n * (NV + 1) * sizeof(hcComplex),
                                   hipMemcpyDeviceToHost));
            HC_HIP_CHECK(hipMemcpy(p->h_conv.data(), p->d_conv, n, hipMemcpyDeviceToHost));
            HC_HIP_CHECK(hipMemcpy(p->h_inf.data(), p->d_inf, n, hipMemcpyDeviceToHost));
            HC_HIP_CHECK(hipMemcpy(p->h_stats.data(), p->d_stats, n * sizeof(hcPathStats), hipMemcpyDeviceToHost));
        }
        if (Abort_RANSAC_by_Good_Sol) {
            HC_HIP_CHECK(hipMemcpy(&p->h_found, p->d_found, 1, hipMemcpyDeviceToHost));
            if (n)
                HC_HIP_CHECK(hipMemcpy(p->h_batch_index.data(), p->d_batch_index, n * sizeof(int32_t),
                                       hipMemcpyDeviceToHost));
            double ff = -1.0;
            hc_trifocal_read_timings(p->d_ws, &ff);
            first_good_pose_time[p->g] = ff;
        }
        transfer_d2h_time[p->g] = now_s() - t0;
        h_GPU_HC_Track_Sols_Stack.insert(h_GPU_HC_Track_Sols_Stack.end(), p->h_track.begin(), p->h_track.end());
        h_is_GPU_HC_Sol_Converge_Stack.insert(h_is_GPU_HC_Sol_Converge_Stack.end(), p->h_conv.begin(), p->h_conv.end());
        h_is_GPU_HC_Sol_Infinity_Stack.insert(h_is_GPU_HC_Sol_Infinity_Stack.end(), p->h_inf.begin(), p->h_inf.end());
        h_Path_Stats_Stack.insert(h_Path_Stats_Stack.end(), p->h_stats.begin(), p->h_stats.end());
        if (Abort_RANSAC_by_Good_Sol) {
            h_Batch_Index_Stack.insert(h_Batch_Index_Stack.end(), p->h_batch_index.begin(), p->h_batch_index.end());
            h_Found_Stack.push_back(p->h_found);
        }
    }

    std::cout << "---------------------------------------------------------------------------------" << std::endl;
    std::cout << "## Solving " << HC_print_problem_name << std::endl << std::endl;
    printf("## Timings:\n");
    printf(" - GPU Computation Time = %7.2f (ms)\n", multi_GPUs_time * 1000);   // :492

    int32_t counts[3] = {0, 0, 0};                                              // :512
    hc_count_solutions(Num_Of_RANSAC_Iterations, reinterpret_cast<const float *>(h_GPU_HC_Track_Sols_Stack.data()),
                       h_is_GPU_HC_Sol_Converge_Stack.data(), h_is_GPU_HC_Sol_Infinity_Stack.data(), counts);
    std::cout << "\n## Evaluation of GPU-HC Solutions: " << std::endl;
    std::cout << " - Number of Converged Solutions:       " << counts[0] << std::endl;
    std::cout << " - Number of Real Solutions:            " << counts[1] << std::endl;
    std::cout << " - Number of Infinity Failed Solutions: " << counts[2] << std::endl;
    Collect_Num_Of_Coverged_Sols.push_back(counts[0]);
    Collect_Num_Of_Real_Sols.push_back(counts[1]);
    Collect_Num_Of_Inf_Sols.push_back(counts[2]);
    {
        std::vector<hcPoseSelection> parts;
        std::vector<int32_t> offs;
        int off = 0;
        for (PerGPU *p : gpus_) {
            parts.push_back(p->h_sel);
            offs.push_back(off);
            off += NT * p->N;
        }
        hc_pose_merge((int)parts.size(), parts.data(), offs.data(), Pose_Flags, &pose_selection);
        pose_success = false;
        for (float &v : pose_residuals) v = -1.0f;
        if (pose_selection.num_candidates > 0) {                                // :490-503
            std::cout << "### Found GT pose!" << std::endl;
            pose_success = hc_pose_residuals(h_Camera_Pose21, h_Camera_Pose31, pose_selection.R21, pose_selection.t21,
                                             pose_selection.R31, pose_selection.t31, pose_residuals) != 0;
        }
        printf("\n## Maximal-support pose (%d candidates, %.3f ms on device):\n", pose_selection.num_candidates,
               pose_time * 1e3);
        printf(" - views 1-2: path %d, %d inliers; views 1-3: path %d, %d inliers\n", pose_selection.path21,
               pose_selection.inliers21, pose_selection.path31, pose_selection.inliers31);
        std::cout << (pose_success ? "## Found solution matched with GT: " : "## Not found a solution matched with GT: ")
                  << std::endl;                                                 // :552-565
        printf(" - Residual of R21: %g (rad)\n - Residual of R31: %g (rad)\n", pose_residuals[0], pose_residuals[1]);
        printf(" - Residual of t21: %g (m)\n - Residual of t31: %g (m)\n", pose_residuals[2], pose_residuals[3]);
        PoseRecord rec;
        rec.success = pose_success ? 1 : 0;
        for (int k = 0; k < 4; k++) rec.residuals[k] = pose_residuals[k];
        rec.path21 = pose_selection.path21;
        rec.path31 = pose_selection.path31;
        rec.num_candidates = pose_selection.num_candidates;
        Collect_Pose.push_back(rec);
    }
    if (Abort_RANSAC_by_Good_Sol) {
        int g = 0;
        for (PerGPU *p : gpus_) {
            std::cout << "GPU id " << p->dev << " found solution? " << (h_Found_Stack[g] ? "Yes" : "No");
            if (h_Found_Stack[g] && first_good_pose_time[p->g] >= 0)
                printf(" (first good pose after %.3f ms on device)", first_good_pose_time[p->g] * 1e3);
            std::cout << std::endl;
            g++;
        }
    }
}

std::vector<int> GPU_HC_Solver::found_batch_ids() const {
    std::vector<int> out;
    for (size_t b = 0; b < h_Batch_Index_Stack.size(); b++)
        if (h_Batch_Index_Stack[b] >= 0) out.push_back((int)b);
    return out;
}

void GPU_HC_Solver::Export_Data() {}

void GPU_HC_Solver::Free_Triplet_Edgels_Mem() {
    h_Triplet_Edge_Locations.clear();
    h_Triplet_Edge_Tangents.clear();
}

void GPU_HC_Solver::Free_Arrays_for_Aborting_RANSAC() {
    // GPU_HC_Solver.cpp:573-587
    if (!Abort_RANSAC_by_Good_Sol) return;
    for (PerGPU *p : gpus_) {
        (void)hipSetDevice(p->dev);
        (void)hipFree(p->d_found);
        (void)hipFree(p->d_batch_index);
        p->d_found = nullptr;
        if (d_peer_found && p == gpus_.front()) {
            (void)hipFree(d_peer_found);
            d_peer_found = nullptr;
        }
        p->d_batch_index = nullptr;
    }
}

GPU_HC_Solver::~GPU_HC_Solver() {
    for (PerGPU *p : gpus_) {
        (void)hipSetDevice(p->dev);
        void *bufs[] = {p->d_Start_Sols, p->d_Track, p->d_Start_Params, p->d_Target_Params, p->d_diffParams,
                        p->d_unified_index, p->d_conv, p->d_inf, p->d_stats, p->d_ws, p->d_edgels, p->d_K,
                        p->d_found, p->d_batch_index, p->d_inliers, p->d_sel};
        for (void *b : bufs)
            if (b) (void)hipFree(b);
        if (p->ev0) (void)hipEventDestroy(p->ev0);
        if (p->ev1) (void)hipEventDestroy(p->ev1);
        if (p->stream) (void)hipStreamDestroy(p->stream);
        delete p;
    }
}

// ------------------------------------------------------------------ CLI driver
bool run_GPU_HC_Solver(const HC_Settings &settings, const std::string &root_dir, int test_ransac_times) {
    // cmd/magmaHC-main.cpp:24-119
    std::vector<double> all_ms;
    GPU_HC_Solver GPU_HC_(settings, root_dir);
    GPU_HC_.Allocate_Arrays();
    for (int ti = 0; ti < test_ransac_times; ti++) {
        if (!GPU_HC_.Read_Problem_Data()) return false;
        if (!GPU_HC_.Read_RANSAC_Data(ti)) return false;
        GPU_HC_.Prepare_Target_Params(ti);
        GPU_HC_.Set_RANSAC_Abort_Arrays();
        GPU_HC_.Data_Transfer_From_Host_To_Device();
        GPU_HC_.Set_CUDA_Stream_Attributes();
        GPU_HC_.Solve_by_GPU_HC();
        GPU_HC_.Free_Triplet_Edgels_Mem();
        GPU_HC_.Free_Arrays_for_Aborting_RANSAC();
        all_ms.push_back(GPU_HC_.multi_GPUs_time * 1000);
    }
    double avg = 0, mx = 0, mn = 1e30;
    for (double v : all_ms) { avg += v; mx = std::max(mx, v); mn = std::min(mn, v); }
    avg /= (double)all_ms.size();
    double sigma = 0;
    for (double v : all_ms) sigma += (v - avg) * (v - avg);
    sigma = std::sqrt(sigma / (double)all_ms.size());
    printf("\n## Running %d rounds of %d RANSAC iterations:\n", test_ransac_times, GPU_HC_.num_samples());
    printf(" - [Average GPU Computation Time] %7.2f (ms)\n", avg);
    printf(" - [Maximal GPU Computation Time] %7.2f (ms)\n", mx);
    printf(" - [Minimal GPU Computation Time] %7.2f (ms)\n", mn);
    printf(" - [Std dev GPU Computation Time] %7.2f (ms)\n", sigma);
    std::string root = root_dir;
    if (!root.empty() && root.back() != '/') root += '/';
    std::error_code ec;
    std::filesystem::create_directories(root + "Output_Write_Files", ec);
    std::ofstream tf(root + "Output_Write_Files/GPU_Timings.txt");
    if (!tf) std::cerr << "cannot write " << root << "Output_Write_Files/GPU_Timings.txt" << std::endl;
    for (double v : all_ms) tf << v << "\n";
    // reference file columns: converged, "inf" (holds real), "real" (holds inf) -- written
    // here with the same byte layout: converged \t real \t inf (cmd/magmaHC-main.cpp:107-116)
    std::ofstream sf(root + "Output_Write_Files/GPU_Sols_Statistics.txt");
    for (size_t i = 0; i < GPU_HC_.Collect_Num_Of_Coverged_Sols.size(); i++)
        sf << GPU_HC_.Collect_Num_Of_Coverged_Sols[i] << "\t" << GPU_HC_.Collect_Num_Of_Real_Sols[i] << "\t"
           << GPU_HC_.Collect_Num_Of_Inf_Sols[i] << "\n";
    // not in the reference: one line per round -- GT match, residuals (rot21 rot31
    // transl21 transl31), selected batch ids, number of candidates
    std::ofstream pf(root + "Output_Write_Files/GPU_Pose_Results.txt");
    for (size_t i = 0; i < GPU_HC_.Collect_Pose.size(); i++) {
        const auto &r = GPU_HC_.Collect_Pose[i];
        pf << r.success << "\t" << r.residuals[0] << "\t" << r.residuals[1] << "\t" << r.residuals[2] << "\t"
           << r.residuals[3] << "\t" << r.path21 << "\t" << r.path31 << "\t" << r.num_candidates << "\n";
    }
    // WRITE_GPUHC_CONVERGED_SOLS (definitions.hpp:22, GPU_HC_Solver.cpp:508-511): last round
    if (settings.b("Write_Converged_Sols", false))
        hc_write_converged_sols((root + "Output_Write_Files/GPU_Converged_HC_tracks.txt").c_str(), GPU_HC_.num_samples(),
                                reinterpret_cast<const float *>(GPU_HC_.tracks().data()), GPU_HC_.converge().data());
    return true;
}
