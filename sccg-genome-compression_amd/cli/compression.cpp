// compression -- drop-in for the reference CLI `compression <reference_file> <target_file>
// <output_folder>` (compression.cpp:584-610): writes <output_folder>/compressed_genome.txt with
// the record stream computed on the GPU (libsccg) and then runs the same 7z command
// (compression.cpp:306-318).  Exit codes follow the reference: 1 on usage / open / 7z errors.
#include "cli_common.h"

#include <cstring>

// Optional, non-parity parameter overrides before the three positional arguments (sccg_params,
// include/sccg.h; the reference hard-codes them at compression.cpp:373-379):
//   --k=<k> --m=<m> --global      (--global: the global pass alone, any 1 <= k <= 32)
static bool parse_option(const std::string& a, sccg_params& p) {
    auto num = [&](const char* pre, int32_t& v) {
        const size_t n = strlen(pre);
        if (a.compare(0, n, pre) != 0) return false;
        char* end = nullptr;
        const long x = strtol(a.c_str() + n, &end, 10);
        if (end == a.c_str() + n || *end) return false;
        v = (int32_t)x;
        return true;
    };
    if (a == "--global") { p.local = 0; return true; }
    return num("--k=", p.k) || num("--m=", p.m);
}

int main(int argc, char* argv[]) {
    sccg_params prm;
    sccg_params_default(&prm);
    int a0 = 1;
    while (a0 < argc && std::string(argv[a0]).compare(0, 2, "--") == 0) {
        if (!parse_option(argv[a0], prm)) {
            std::cerr << "Unknown option: " << argv[a0] << "\n";
            return 1;
        }
        a0++;
    }
    if (argc - a0 != 3) {
        std::cerr << "Usage: " << argv[0] << " [--k=K --m=M --global] <reference_file> <target_file> <output_folder>\n";
        return 1;
    }
    const std::string ref_path = argv[a0], tgt_path = argv[a0 + 1], out_dir = argv[a0 + 2];
    try {
        if (!std::filesystem::exists(out_dir)) std::filesystem::create_directory(out_dir);
    } catch (const std::exception& ex) {
        std::cerr << "Error: " << ex.what() << "\n";
        return 1;
    }
    std::cout << "Successfully created output folder: " << out_dir << "\n";
    const auto t0 = std::chrono::high_resolution_clock::now();
    sccg_ctx* ctx = nullptr;
    int rc = sccg_ctx_create(cli_device(), &ctx);
    if (rc) {
        std::cerr << "Error: no usable GPU (sccg_ctx_create rc=" << rc << ")\n";
        return 1;
    }
    // files -> record file in the library (pinned staging, reads overlapped with the GPU work)
    std::filesystem::create_directories(out_dir);
    const std::string txt = out_dir + "/compressed_genome.txt";
    rc = sccg_compress_files(ctx, &prm, ref_path.c_str(), tgt_path.c_str(), txt.c_str(), nullptr);
    if (rc == SCCG_E_OPEN_REF || rc == SCCG_E_OPEN_TGT) {   // compression.cpp:189 / :204
        std::cerr << (rc == SCCG_E_OPEN_REF ? "Error opening reference file: " : "Error opening target file: ")
                  << (rc == SCCG_E_OPEN_REF ? ref_path : tgt_path) << "\n";
        sccg_ctx_destroy(ctx);
        return 1;
    }
    if (rc == SCCG_E_WRITE) {
        std::cerr << "Greska pri otvaranju datoteke: " << txt << "\n";
        sccg_ctx_destroy(ctx);
        return 1;
    }
    if (rc && rc != SCCG_E_DELTA_STOI) {
        std::cerr << "Error: " << sccg_last_error(ctx) << " (rc=" << rc << ")\n";
        sccg_ctx_destroy(ctx);
        return 1;
    }
    sccg_stats st{};
    sccg_last_stats(ctx, &st);
    sccg_ctx_destroy(ctx);
    if (rc == SCCG_E_DELTA_STOI) {   // the reference throws from stoi inside delta_encode
        std::cerr << "Error: stoi\n";
        return 1;
    }
    std::cout << "mode=" << (st.mode_global ? "global" : "local") << " switch=" << st.switch_segment
              << " matches=" << st.n_matches << " bytes=" << st.record_bytes << "\n";
    const int r = run_argv({"7z", "a", "-mx=9", txt + ".7z", txt});   // compression.cpp:308
    if (r != 0) {
        std::cerr << "Greska prilikom komprimiranja datoteke 7-zipom: " << r << " !\n";
        return 1;
    }
    const std::chrono::duration<double> dt = std::chrono::high_resolution_clock::now() - t0;
    std::cout << "Time taken to compress: " << dt.count() << " s\n";
    return 0;
}
