// magmaHC-main -- CLI of the MI355X GPU-HC tracker, surface-compatible with the
// reference's build/bin/magmaHC-main (cmd/magmaHC-main.cpp:197-260):
//
//   magmaHC-main -p trifocal_2op1p_30x30 [-d <repository root>] [-n <RANSAC samples>]
//                [-g <num GPUs>] [-t <test rounds>] [--abort]
//
// Reads <root>/problems/<problem>/gpuhc_settings.yaml (falls back to
// <root>/data/problems/...), runs GPU-HC and the device pose recovery, writes
// GPU_Timings.txt, GPU_Sols_Statistics.txt, GPU_Pose_Results.txt (and with
// --write-sols GPU_Converged_HC_tracks.txt) under <root>/Output_Write_Files/.  The root defaults
// to "../../" like the reference binary (run from <repo>/<pkg>/bin).
#include <cstdio>
#include <exception>
#include <fstream>
#include <iostream>
#include <string>

#include "../../include/GPU_HC_Solver.hpp"

static void usage() {
    printf("Usage: ./magmaHC-main [options] [path]\n\n"
           "options:\n"
           "  -h, --help        show this help message and exit\n"
           "  -p, --problem     problem name, e.g. trifocal_2op1p_30x30\n"
           "  -d, --directory   repository directory (default ../../)\n"
           "  -n, --samples     RANSAC samples per run (NUM_OF_RANSAC_ITERATIONS, default 100)\n"
           "  -g, --gpus        number of GPUs (overrides Num_Of_GPUs)\n"
           "  -t, --times       test rounds (TEST_RANSAC_TIMES, default 1)\n"
           "      --abort       Abort_RANSAC_by_Good_Sol = true\n"
           "      --share-devices  allow more GPUs (-g) than devices: logical GPU g runs on device g %% count\n"
           "      --inflight-stop  abort mode: paths in flight also stop once a pose is found\n"
           "                    (Abort_Inflight_Stop; default: they run to completion as in the reference)\n"
           "      --abort-across-gpus  abort mode: one found flag shared by all GPUs (Abort_Across_GPUs;\n"
           "                    default: one flag per GPU as in the reference)\n"
           "      --write-sols  write Output_Write_Files/GPU_Converged_HC_tracks.txt\n"
           "      --quirks      reference-literal pose selection (Pose_Selection_Reference_Quirks)\n"
           "  -s, --dataset     RANSAC dataset directory name (default Synthetic)\n");
}

int main(int argc, char **argv) {
    std::string problem, root = "../../";
    int samples = -1, gpus = -1, times = 1;
    bool abort_flag = false, write_sols = false, quirks = false, inflight_stop = false, share = false,
         across = false;
    std::string dataset;
    if (argc <= 1) { usage(); return 0; }
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&](const char *what) -> std::string {
            if (i + 1 >= argc) { printf("\033[1;31m[ERROR] missing value for %s\033[0m\n", what); usage(); exit(0); }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (a == "-p" || a == "--problem") problem = next("-p");
        else if (a == "-d" || a == "--directory") root = next("-d");
        else if (a == "-n" || a == "--samples") samples = std::stoi(next("-n"));
        else if (a == "-g" || a == "--gpus") gpus = std::stoi(next("-g"));
        else if (a == "-t" || a == "--times") times = std::stoi(next("-t"));
        else if (a == "--abort") abort_flag = true;
        else if (a == "--inflight-stop") inflight_stop = true;
        else if (a == "--abort-across-gpus") across = true;
        else if (a == "--share-devices") share = true;
        else if (a == "--write-sols") write_sols = true;
        else if (a == "--quirks") quirks = true;
        else if (a == "-s" || a == "--dataset") dataset = next("-s");
        else { printf("\033[1;31m[ERROR] Invalid input arguments!\033[0m\n"); usage(); return 0; }
    }
    if (problem.empty()) { usage(); return 0; }
    if (!root.empty() && root.back() != '/') root += '/';
    std::string yaml = root + "problems/" + problem + "/gpuhc_settings.yaml";
    if (!std::ifstream(yaml)) yaml = root + "data/problems/" + problem + "/gpuhc_settings.yaml";
    try {
        HC_Settings s = HC_Settings::LoadFile(yaml);
        for (const auto &kv : s.items()) std::cout << kv.first << ": " << kv.second << "\n";
        std::cout << std::endl;
        if (samples > 0) s.set("Num_Of_RANSAC_Iterations", std::to_string(samples));
        if (gpus > 0) s.set("Num_Of_GPUs", std::to_string(gpus));
        if (abort_flag) s.set("Abort_RANSAC_by_Good_Sol", "true");
        if (inflight_stop) s.set("Abort_Inflight_Stop", "true");
        if (across) s.set("Abort_Across_GPUs", "true");
        if (share) s.set("Share_Devices", "true");
        if (write_sols) s.set("Write_Converged_Sols", "true");
        if (quirks) s.set("Pose_Selection_Reference_Quirks", "true");
        if (!dataset.empty()) s.set("RANSAC_Dataset", dataset);
        if (!run_GPU_HC_Solver(s, root, times)) return 1;
    } catch (const std::exception &e) {
        std::cerr << "Exception: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
