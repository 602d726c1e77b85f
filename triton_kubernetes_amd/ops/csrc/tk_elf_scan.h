// Find an exported RCCL device-kernel handle by scanning a shared library's dynamic symbol
// table, instead of trusting one mangled name.
//
// tkr_preload_device_code (tk_rccl_probe.hip) triggers the load of librccl's device code
// by querying the attributes of one kernel the library exports.  Which kernels are exported,
// and under which mangled names, depends on the build: /opt/rocm's librccl (ROCm 7.2)
// exports `ncclDevKernel_Generic_{1,2,4}` as data symbols (HIP host-side kernel handles),
// the librccl torch ships exports `rcclGenericKernel<N, bool>` as weak objects instead
// (tests/test_burnin_policy.py checks both on this image).  Every RCCL device kernel takes
// an `ncclDevKernelArgsStorage<...>`, so that type's mangled name is the needle; the debug
// variants are skipped.
//
// Pure ELF reading (mmap, bounds-checked): no HIP, so the stub library and a CPU test use
// the same scanner.

#pragma once

#include <elf.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <string>

// The first defined dynamic symbol of the ELF64 file at `path` whose name contains
// `needle` and not `reject` (nullptr: none); "" when there is none or the file is unreadable.
static inline std::string tk_elf_find_symbol(const char* path, const char* needle, const char* reject) {
  std::string found;
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return found;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < (off_t)sizeof(Elf64_Ehdr)) {
    close(fd);
    return found;
  }
  const size_t size = (size_t)st.st_size;
  void* map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (map == MAP_FAILED) return found;
  const unsigned char* base = (const unsigned char*)map;
  auto in_file = [size](uint64_t off, uint64_t len) { return off <= size && len <= size - off; };
  const Elf64_Ehdr* eh = (const Elf64_Ehdr*)base;
  if (memcmp(eh->e_ident, ELFMAG, SELFMAG) == 0 && eh->e_ident[EI_CLASS] == ELFCLASS64 &&
      eh->e_shentsize == sizeof(Elf64_Shdr) && in_file(eh->e_shoff, (uint64_t)eh->e_shnum * sizeof(Elf64_Shdr))) {
    const Elf64_Shdr* sh = (const Elf64_Shdr*)(base + eh->e_shoff);
    for (int i = 0; i < eh->e_shnum && found.empty(); ++i) {
      if (sh[i].sh_type != SHT_DYNSYM || sh[i].sh_link >= eh->e_shnum) continue;
      const Elf64_Shdr& strs = sh[sh[i].sh_link];
      if (!in_file(sh[i].sh_offset, sh[i].sh_size) || !in_file(strs.sh_offset, strs.sh_size)) continue;
      const Elf64_Sym* syms = (const Elf64_Sym*)(base + sh[i].sh_offset);
      const char* names = (const char*)(base + strs.sh_offset);
      const size_t nsym = sh[i].sh_size / sizeof(Elf64_Sym);
      for (size_t k = 1; k < nsym; ++k) {
        const Elf64_Sym& s = syms[k];
        const int type = ELF64_ST_TYPE(s.st_info);
        if (s.st_shndx == SHN_UNDEF || (type != STT_OBJECT && type != STT_FUNC)) continue;
        if (s.st_name >= strs.sh_size) continue;
        const char* name = names + s.st_name;
        const size_t room = strs.sh_size - s.st_name;
        if (strnlen(name, room) == room) continue;  // not terminated inside the table
        if (strstr(name, needle) && !(reject && strstr(name, reject))) {
          found = name;
          break;
        }
      }
    }
  }
  munmap(map, size);
  return found;
}

// The kernel-handle needle and the variants skipped (see the header comment).
static constexpr const char* kTkRcclKernelNeedle = "ncclDevKernelArgsStorage";
static constexpr const char* kTkRcclKernelReject = "Debug";
