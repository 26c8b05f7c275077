// Small procfs / sysfs / cgroupfs readers shared by the native samplers (procsampler, gpusampler).
#pragma once

#include <fcntl.h>
#include <unistd.h>

#include <cstdint>
#include <cstdlib>
#include <string>

namespace mislo {

// Whole small file into `out` (procfs / sysfs files are a page at most). False if unreadable.
inline bool read_small(const std::string& path, std::string* out) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  char buf[4096];
  out->clear();
  for (;;) {
    const ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0) {
      ::close(fd);
      return false;
    }
    if (n == 0) break;
    out->append(buf, (size_t)n);
    if (out->size() > (1u << 16)) break;
  }
  ::close(fd);
  return true;
}

// A file holding one decimal number (sysfs attributes). False if unreadable or empty.
inline bool read_u64_file(const char* path, uint64_t* v) {
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  char buf[32];
  const ssize_t n = ::read(fd, buf, sizeof(buf) - 1);
  ::close(fd);
  if (n <= 0) return false;
  buf[n] = 0;
  *v = std::strtoull(buf, nullptr, 10);
  return true;
}

// The same from a file kept open: one pread at offset 0 (sysfs regenerates the attribute on
// every read from the start), no open / close per reading.
inline bool pread_u64(int fd, uint64_t* v) {
  char buf[32];
  const ssize_t n = ::pread(fd, buf, sizeof(buf) - 1, 0);
  if (n <= 0) return false;
  buf[n] = 0;
  *v = std::strtoull(buf, nullptr, 10);
  return true;
}

inline std::string join(const std::string& a, const std::string& b) {
  std::string r = a;
  while (!r.empty() && r.back() == '/') r.pop_back();
  size_t i = 0;
  while (i < b.size() && b[i] == '/') ++i;
  if (i == b.size()) return r.empty() ? std::string("/") : r;
  return r + "/" + b.substr(i);
}

// The process's pid in its own (innermost) pid namespace: the last NSpid field.
inline uint32_t ns_pid_of(const std::string& proc_root, uint32_t pid) {
  std::string s;
  if (!read_small(join(proc_root, std::to_string(pid) + "/status"), &s)) return pid;
  const size_t k = s.find("\nNSpid:");
  if (k == std::string::npos) return pid;
  size_t e = s.find('\n', k + 1);
  if (e == std::string::npos) e = s.size();
  size_t end = e;
  while (end > k && (s[end - 1] == ' ' || s[end - 1] == '\t')) --end;
  size_t beg = end;
  while (beg > k && s[beg - 1] != ' ' && s[beg - 1] != '\t' && s[beg - 1] != ':') --beg;
  if (beg >= end) return pid;
  return (uint32_t)std::strtoul(s.c_str() + beg, nullptr, 10);
}

}  // namespace mislo
