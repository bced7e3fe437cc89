// cli_common.h -- shared helpers of the reference-compatible command lines.
#pragma once
#include <sccg.h>

#include <chrono>
#include <cstdio>
#include <cerrno>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include <spawn.h>
#include <sys/wait.h>

extern char** environ;

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

// The reference runs 7z through std::system with the paths pasted into a shell string
// (compression.cpp:308, decompression.cpp:34).  Same command, same stdout/stderr, same status
// word (the wait status, as std::system returns it; 127 << 8 when 7z cannot be started, as the
// shell reports it), but as an argv list: a path holding '"', '$(' or '`' is passed as a path,
// never interpreted by a shell.
inline int run_argv(const std::vector<std::string>& args) {
    std::vector<char*> av;
    for (const std::string& a : args) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    std::cout.flush();
    pid_t pid = 0;
    if (posix_spawnp(&pid, av[0], nullptr, nullptr, av.data(), environ) != 0) return 127 << 8;
    int status = 0;
    while (waitpid(pid, &status, 0) < 0) {
        if (errno != EINTR) return -1;
    }
    return status;
}
