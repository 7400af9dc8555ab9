// GPU_HC_Solver.hpp -- C++ host driver of the MI355X GPU-HC tracker.
//
// Keeps the public surface of the reference class (magmaHC/GPU_HC_Solver.hpp:98-120)
// so the reference's RANSAC driver (cmd/magmaHC-main.cpp:24-119) drops in:
//   ctor(settings), Allocate_Arrays, Read_Problem_Data, Read_RANSAC_Data(int),
//   Prepare_Target_Params(unsigned), Set_RANSAC_Abort_Arrays,
//   Data_Transfer_From_Host_To_Device, Set_CUDA_Stream_Attributes (no-op on
//   CDNA: the compacted index tables live in LDS), Solve_by_GPU_HC,
//   Free_Triplet_Edgels_Mem, Free_Arrays_for_Aborting_RANSAC, the timers and
//   the Collect_* statistics vectors.
// Underneath, every launch goes through the C-ABI of include/hc_trifocal.h;
// MAGMA / CUDA / yaml-cpp are not used.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "hc_pose.h"
#include "hc_trifocal.h"

#define MAX_NUM_OF_GPUS 8   // definitions.hpp:8

// Flat `key: value` view of gpuhc_settings.yaml (stands in for YAML::Node).
class HC_Settings {
public:
    HC_Settings() = default;
    static HC_Settings LoadFile(const std::string &path);   // throws std::runtime_error
    bool has(const std::string &k) const { return kv_.count(k) != 0; }
    std::string str(const std::string &k) const;
    int i(const std::string &k, int dflt) const;
    bool b(const std::string &k, bool dflt) const;
    void set(const std::string &k, const std::string &v) { kv_[k] = v; }
    const std::map<std::string, std::string> &items() const { return kv_; }

private:
    std::map<std::string, std::string> kv_;
};

class GPU_HC_Solver {
public:
    // timers (seconds): gpu_time[g] = device time of GPU g's launch (HIP events),
    // multi_GPUs_time = host wall time launch -> all GPUs synchronised
    // (GPU_HC_Solver.cpp:384,446 scope)
    double gpu_time[MAX_NUM_OF_GPUS] = {0.0};
    double transfer_h2d_time[MAX_NUM_OF_GPUS] = {0.0};
    double transfer_d2h_time[MAX_NUM_OF_GPUS] = {0.0};
    double multi_GPUs_time = 0.0;
    double first_good_pose_time[MAX_NUM_OF_GPUS] = {0.0};   // abort mode, device clock (s), <0: none
    double pose_time = 0.0;   // device pose recovery + maximal support, all GPUs (s)

    // maximal-support pose of the last run (Evaluations.cpp:298-543 on the device,
    // include/hc_pose.h) and its error against GT_Poses21/31 of the data index
    hcPoseSelection pose_selection{};
    float pose_residuals[4] = {-1.0f, -1.0f, -1.0f, -1.0f};   // rot21, rot31 (rad), transl21, transl31
    bool pose_success = false;
    struct PoseRecord {
        int success = 0;
        float residuals[4] = {-1.0f, -1.0f, -1.0f, -1.0f};
        int path21 = -1, path31 = -1, num_candidates = 0;
    };
    std::vector<PoseRecord> Collect_Pose;   // one per Solve_by_GPU_HC

    explicit GPU_HC_Solver(const HC_Settings &settings, const std::string &root_dir = "../../");
    ~GPU_HC_Solver();

    bool Read_Problem_Data();
    bool Read_RANSAC_Data(int tp_index);
    void Allocate_Arrays();
    void Prepare_Target_Params(unsigned rand_seed_);
    void Data_Transfer_From_Host_To_Device();
    void Set_CUDA_Stream_Attributes();
    void Set_RANSAC_Abort_Arrays();
    void Solve_by_GPU_HC();
    void Export_Data();
    void Free_Triplet_Edgels_Mem();
    void Free_Arrays_for_Aborting_RANSAC();

    // Evaluations::Evaluate_RANSAC_HC_Sols results per run (correct names; the
    // reference fills the inf / real vectors swapped, GPU_HC_Solver.cpp:522-524)
    std::vector<unsigned> Collect_Num_Of_Coverged_Sols;
    std::vector<unsigned> Collect_Num_Of_Inf_Sols;
    std::vector<unsigned> Collect_Num_Of_Real_Sols;

    // results of the last Solve_by_GPU_HC, stacked over GPUs in sample order
    const std::vector<hcComplex> &tracks() const { return h_GPU_HC_Track_Sols_Stack; }
    const std::vector<uint8_t> &converge() const { return h_is_GPU_HC_Sol_Converge_Stack; }
    const std::vector<uint8_t> &infinity() const { return h_is_GPU_HC_Sol_Infinity_Stack; }
    const std::vector<hcPathStats> &path_stats() const { return h_Path_Stats_Stack; }
    std::vector<int> found_batch_ids() const;   // abort mode: batch ids of passing hypotheses
    int num_samples() const { return Num_Of_RANSAC_Iterations; }
    int num_gpus() const { return Num_Of_GPUs; }
    bool abort_mode() const { return Abort_RANSAC_by_Good_Sol; }

private:
    struct PerGPU;
    std::vector<PerGPU *> gpus_;

    // settings (GPU_HC_Solver.cpp:46-66)
    std::string HC_problem, HC_print_problem_name, RANSAC_Dataset_Name;
    int GPUHC_Max_Steps = 80, GPUHC_Max_Correction_Steps = 3, GPUHC_delta_t_incremental_steps = 4;
    int Num_Of_Vars = 30, Num_Of_Params = 33, Num_Of_Tracks = 312;
    bool Abort_RANSAC_by_Good_Sol = false;
    bool Abort_Inflight_Stop = false;   // not in the reference: hcAbortArgs::inflight_stop
    bool Abort_Across_GPUs = false;     // not in the reference: one found flag for all GPUs (hcAbortArgs::peer_found)
    uint32_t *d_peer_found = nullptr;   // on the first GPU's device, read and set by every GPU's launch
    const char *peer_flag_kind_ = nullptr;   // memory the flag got: "uncached", "fine-grained" or "coarse-grained (hipMalloc)"
    int Pose_Flags = 0;   // Pose_Selection_Reference_Quirks -> HC_POSE_REFERENCE_QUIRKS
    int Num_Of_GPUs = 1;
    int Num_Of_RANSAC_Iterations = 100;   // NUM_OF_RANSAC_ITERATIONS (definitions.hpp:12), runtime here
    int sub_RANSAC_iters[MAX_NUM_OF_GPUS] = {0};
    std::string Problem_File_Path, RANSAC_Data_File_Path, Write_Files_Path;

    // host data
    std::vector<float> h_Start_Sols, h_Start_Params, h_Target_Params, h_diffParams;
    std::vector<int32_t> h_unified_dHdx_dHdt_Index;
    std::vector<float> h_Triplet_Edge_Locations, h_Triplet_Edge_Tangents;
    float h_Camera_Intrinsic_Matrix[9] = {0};
    float h_Camera_Pose21[12] = {0}, h_Camera_Pose31[12] = {0};
    int Num_Of_Triplet_Edgels = 0;
    std::vector<int32_t> h_picked;

    std::vector<hcComplex> h_GPU_HC_Track_Sols_Stack;
    std::vector<uint8_t> h_is_GPU_HC_Sol_Converge_Stack, h_is_GPU_HC_Sol_Infinity_Stack;
    std::vector<hcPathStats> h_Path_Stats_Stack;
    std::vector<int32_t> h_Batch_Index_Stack;
    std::vector<uint8_t> h_Found_Stack;
};

// CLI helpers shared by magmaHC-main and tests
bool run_GPU_HC_Solver(const HC_Settings &settings, const std::string &root_dir, int test_ransac_times);
