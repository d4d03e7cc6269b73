// selfcheck.hpp — host-only: does this library's gfx950 code object hold every kernel its host code launches?
//
// A HIP launch of a kernel whose device symbol is absent from the loaded code object does not return an
// error: the runtime aborts the process ("Cannot find Symbol with name: ...", hip_global.cpp).  That
// happened once in round 5 with an experiment build (DESIGN.md §4 "Load-time kernel check"): hipcc compiles
// the device pass and the host pass of a source separately, and a source edited between the two passes gave
// host stubs for a kernel the device pass had never seen.  This check turns that into an error the
// caller sees before any launch.
//
// It reads the library's own file (dladdr of a symbol in it) and compares two lists:
//   host side   every kernel handle the host code registers: for each `__device_stub__` function symbol of
//               the ELF symbol table, the mangled kernel name it stands for (the stub's mangled name with
//               "<n>__device_stub__" replaced by "<n - 15>");
//   device side the kernel descriptors (`<name>.kd`) in the symbol table of the gfx950 code object inside
//               the `.hip_fatbin` section (a clang offload bundle).
// Every host name must have a device descriptor.  Pure file parsing: no HIP call, so it also runs on a
// machine without a GPU (tests/test_native_abi.py checks a clean and a deliberately broken library).
#pragma once
#include <dlfcn.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <set>
#include <string>
#include <vector>

namespace wd {

namespace elfchk {

struct Shdr { uint32_t name, type; uint64_t flags, addr, off, size; uint32_t link, info; uint64_t align, entsize; };

inline bool rd_shdrs(const std::vector<uint8_t> &f, size_t base, size_t len, std::vector<Shdr> &out, size_t &shstr) {
    if (len < 64 || memcmp(f.data() + base, "\x7f" "ELF", 4) != 0 || f[base + 4] != 2) return false;  // ELF64 only
    uint64_t shoff;
    uint16_t shentsize, shnum, shstrndx;
    memcpy(&shoff, f.data() + base + 0x28, 8);
    memcpy(&shentsize, f.data() + base + 0x3a, 2);
    memcpy(&shnum, f.data() + base + 0x3c, 2);
    memcpy(&shstrndx, f.data() + base + 0x3e, 2);
    if (shentsize != 64 || shoff + (uint64_t)shnum * 64 > len || shstrndx >= shnum) return false;
    out.resize(shnum);
    for (int i = 0; i < shnum; ++i) {
        const uint8_t *p = f.data() + base + shoff + 64 * (size_t)i;
        Shdr &s = out[i];
        memcpy(&s.name, p, 4); memcpy(&s.type, p + 4, 4); memcpy(&s.flags, p + 8, 8); memcpy(&s.addr, p + 16, 8);
        memcpy(&s.off, p + 24, 8); memcpy(&s.size, p + 32, 8); memcpy(&s.link, p + 40, 4); memcpy(&s.info, p + 44, 4);
        memcpy(&s.align, p + 48, 8); memcpy(&s.entsize, p + 56, 8);
        if (s.type != 8 /* NOBITS */ && s.off + s.size > len) return false;
    }
    shstr = out[shstrndx].off;
    return true;
}

inline std::string cstr(const std::vector<uint8_t> &f, size_t at, size_t end) {
    size_t e = at;
    while (e < end && f[e]) ++e;
    return std::string(reinterpret_cast<const char *>(f.data() + at), e - at);
}

// names of the symbols of the first SHT_SYMTAB (2) section, or of SHT_DYNSYM (11) when there is none
inline bool symbols(const std::vector<uint8_t> &f, size_t base, size_t len, std::vector<std::string> &names) {
    std::vector<Shdr> sh;
    size_t shstr;
    if (!rd_shdrs(f, base, len, sh, shstr)) return false;
    int pick = -1;
    for (int want : {2, 11}) {
        for (size_t i = 0; i < sh.size() && pick < 0; ++i)
            if ((int)sh[i].type == want) pick = (int)i;
        if (pick >= 0) break;
    }
    if (pick < 0 || sh[pick].link >= sh.size()) return false;
    const Shdr &st = sh[pick], &ss = sh[st.link];
    for (size_t o = 0; o + 24 <= st.size; o += 24) {
        uint32_t nm;
        memcpy(&nm, f.data() + base + st.off + o, 4);
        if (nm) names.push_back(cstr(f, base + ss.off + nm, base + ss.off + ss.size));
    }
    return true;
}

inline bool section(const std::vector<uint8_t> &f, const char *want, size_t &off, size_t &size) {
    std::vector<Shdr> sh;
    size_t shstr;
    if (!rd_shdrs(f, 0, f.size(), sh, shstr)) return false;
    for (const Shdr &s : sh)
        if (cstr(f, shstr + s.name, f.size()) == want) { off = s.off; size = s.size; return true; }
    return false;
}

// the kernel a host stub symbol stands for ("" if the name is not a stub)
inline std::string stub_kernel(const std::string &s) {
    static const char tag[] = "__device_stub__";
    const size_t at = s.find(tag);
    if (at == std::string::npos || s.compare(0, 2, "_Z") != 0) return "";
    size_t d = at;
    while (d > 0 && s[d - 1] >= '0' && s[d - 1] <= '9') --d;
    if (d == at) return "";
    const int n = atoi(s.substr(d, at - d).c_str()) - (int)(sizeof(tag) - 1);
    if (n <= 0) return "";
    return s.substr(0, d) + std::to_string(n) + s.substr(at + sizeof(tag) - 1);
}

}  // namespace elfchk

// 0: every registered kernel is in the gfx950 code object; otherwise a message in `why`
inline int code_object_check(const void *addr_in_lib, std::string &why, int &n_host, int &n_dev) {
    using namespace elfchk;
    n_host = n_dev = 0;
    Dl_info di;
    if (!dladdr(addr_in_lib, &di) || !di.dli_fname) { why = "dladdr found no file for the library"; return 1; }
    FILE *fp = fopen(di.dli_fname, "rb");
    if (!fp) { why = std::string("cannot read ") + di.dli_fname; return 1; }
    std::vector<uint8_t> f;
    uint8_t buf[1 << 16];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), fp)) > 0) f.insert(f.end(), buf, buf + got);
    fclose(fp);
    std::vector<std::string> host_syms;
    if (!symbols(f, 0, f.size(), host_syms)) { why = std::string(di.dli_fname) + ": no ELF symbol table"; return 1; }
    std::set<std::string> host;
    for (const std::string &s : host_syms) {
        const std::string k = stub_kernel(s);
        if (!k.empty()) host.insert(k);
    }
    size_t fo, fs;
    if (!section(f, ".hip_fatbin", fo, fs)) { why = std::string(di.dli_fname) + ": no .hip_fatbin section"; return 1; }
    // clang offload bundle: magic, entry count, then per entry {offset, size, triple length, triple}
    static const char magic[] = "__CLANG_OFFLOAD_BUNDLE__";
    std::set<std::string> dev;
    bool found = false;
    for (size_t b = fo; b + 32 <= fo + fs; ) {
        if (memcmp(f.data() + b, magic, 24) != 0) break;
        uint64_t n;
        memcpy(&n, f.data() + b + 24, 8);
        size_t p = b + 32, bundle_end = b;
        for (uint64_t e = 0; e < n && p + 24 <= fo + fs; ++e) {
            uint64_t off, size, tl;
            memcpy(&off, f.data() + p, 8); memcpy(&size, f.data() + p + 8, 8); memcpy(&tl, f.data() + p + 16, 8);
            p += 24;
            const std::string triple = cstr(f, p, p + tl);
            p += tl;
            bundle_end = std::max(bundle_end, (size_t)(b + off + size));
            if (triple.find("gfx950") == std::string::npos || b + off + size > fo + fs) continue;
            std::vector<std::string> ds;
            if (!symbols(f, b + off, size, ds)) { why = "gfx950 code object without a symbol table"; return 1; }
            found = true;
            for (const std::string &s : ds)
                if (s.size() > 3 && s.compare(s.size() - 3, 3, ".kd") == 0) dev.insert(s.substr(0, s.size() - 3));
        }
        // (a fat binary may hold several bundles, each 4 KB aligned)
        size_t next = (bundle_end + 4095) & ~(size_t)4095;
        if (next <= b) break;
        b = next;
    }
    if (!found) { why = "no gfx950 code object in .hip_fatbin"; return 1; }
    n_host = (int)host.size();
    n_dev = (int)dev.size();
    int missing = 0;
    for (const std::string &k : host)
        if (!dev.count(k)) {
            if (missing++ == 0) why = "kernel(s) registered by the host code but absent from the gfx950 code object: " + k;
        }
    if (missing > 1) why += " (+" + std::to_string(missing - 1) + " more)";
    if (missing) why += "; the library's device and host passes were built from different sources: rebuild it";
    return missing ? 1 : 0;
}

}  // namespace wd
