// decompression -- drop-in for the reference CLI `decompression <compressed_file>
// <reference_file> <output_folder>` (decompression.cpp:281-330): runs the same `7z e`
// (decompression.cpp:34), rebuilds the target on the GPU (libsccg) and writes
// <output_folder>/reconstructed_genome.fa.  Exit code 1 on usage / 7z / open / format errors.
#include "cli_common.h"

int main(int argc, char* argv[]) {
    if (argc != 4) {
        std::cerr << "Usage: " << argv[0] << " <compressed_file> <reference_file> <output_folder>\n";
        return 1;
    }
    const std::string arc = argv[1], ref_path = argv[2], out_dir = argv[3];
    const auto t0 = std::chrono::high_resolution_clock::now();
    try {
        if (!std::filesystem::exists(out_dir)) std::filesystem::create_directory(out_dir);
    } catch (const std::exception& ex) {
        std::cerr << "Error: " << ex.what() << "\n";
        return 1;
    }
    if (run_argv({"7z", "e", arc, "-o" + out_dir, "-y"}) != 0) {   // decompression.cpp:34
        std::cerr << "Greska pri dekompresiji: " << arc << "\n";
        return 1;
    }
    const std::string rec_path = out_dir + "/" + std::filesystem::path(arc).stem().string();
    std::string ref, rec;
    if (!slurp(ref_path, ref)) {
        std::cerr << "Greska pri otvaranju reference: " << ref_path << "\n";
        return 1;
    }
    if (!slurp(rec_path, rec)) {
        std::cerr << "Greska pri otvaranju datoteke: " << rec_path << "\n";
        return 1;
    }
    sccg_ctx* ctx = nullptr;
    int rc = sccg_ctx_create(cli_device(), &ctx);
    if (rc) {
        std::cerr << "Error: no usable GPU (sccg_ctx_create rc=" << rc << ")\n";
        return 1;
    }
    sccg_buf fa{};
    rc = sccg_reconstruct(ctx, ref.data(), ref.size(), rec.data(), rec.size(), &fa);
    if (rc) {
        std::cerr << "Error during reconstruction: " << sccg_last_error(ctx) << " (rc=" << rc << ")\n";
        sccg_ctx_destroy(ctx);
        return 1;
    }
    sccg_ctx_destroy(ctx);
    const std::chrono::duration<double> dt = std::chrono::high_resolution_clock::now() - t0;
    const std::string out = out_dir + "/reconstructed_genome.fa";
    if (!spit(out, fa.data, fa.len)) {
        std::cerr << "Error opening output file: " << out_dir << "\n";
        return 1;
    }
    std::cout << "Reconstructed genome written (" << fa.len << " characters) to: " << out_dir << "\n";
    std::cout << "Time taken to decompress: " << dt.count() << " s\n";
    sccg_buf_free(&fa);
    return 0;
}
