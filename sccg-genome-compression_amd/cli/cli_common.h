// cli_common.h -- shared helpers of the reference-compatible command lines.
#pragma once
#include <sccg.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

inline bool slurp(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

inline bool spit(const std::string& path, const char* data, size_t n) {
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f.is_open()) return false;
    f.write(data, (std::streamsize)n);
    return (bool)f;
}

// device index: SCCG_DEVICE, else LOCAL_RANK, else 0
inline int cli_device() {
    const char* e = std::getenv("SCCG_DEVICE");
    if (!e) e = std::getenv("LOCAL_RANK");
    return e ? std::atoi(e) : 0;
}
