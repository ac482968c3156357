// dmf_io.hip — persistent form of the fused log-odds grid (optional
// checkpoint/resume).  Host code only (no GPU needed).  The file holds the FINAL clamped
// int16 grid (what the reference's consumers read), not the int32 hit/miss counters: it is a
// dump of a finished fusion, from which a new fusion cannot resume exactly (clamped log-odds
// do not accumulate; keep the counters for that).
//
// The reference's only persistent outputs are text files (writeCameraLocations,
// FileRoutines.hpp:98-112, and a PCD); the fusion grid it never had.  The file is a
// fixed little-endian header, the int16 grid in the reference's x-major voxel order, and a
// CRC-32 of header + grid, so a torn or foreign file is rejected instead of loaded:
//   "DMFGRID1" | u32 version = 1 | u32 header bytes = 104 | i32 dims[3] | u32 reserved = 0 |
//   f64 bounds[6] (xmin, xmax, ymin, ymax, zmin, zmax) | i32 fuse params[6] | i16 grid[x*y*z] |
//   u32 crc32 (IEEE 802.3, reflected 0xEDB88320) of every byte before it
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "dmf_host.hpp"

namespace dmf {
namespace {

constexpr char kMagic[8] = {'D', 'M', 'F', 'G', 'R', 'I', 'D', '1'};
constexpr uint32_t kVersion = 1, kHeaderBytes = 104;
static_assert(sizeof(dmf_fuse_params) == 24, "six int32 fuse parameters");

struct Crc32 {
  uint32_t table[256];
  Crc32() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = c & 1u ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
  }
  uint32_t update(uint32_t crc, const void* data, size_t n) const {
    const uint8_t* p = (const uint8_t*)data;
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xffu] ^ (crc >> 8);
    return ~crc;
  }
};

const Crc32& crc32() {
  static const Crc32 c;
  return c;
}

void put_header(const dmf_grid_header* h, uint8_t out[kHeaderBytes]) {
  memset(out, 0, kHeaderBytes);
  memcpy(out, kMagic, 8);
  memcpy(out + 8, &kVersion, 4);
  memcpy(out + 12, &kHeaderBytes, 4);
  memcpy(out + 16, h->dims, 12);  // bytes 28..31: reserved (0)
  memcpy(out + 32, h->bounds, 48);
  memcpy(out + 80, &h->params, 24);
}

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) fclose(f);
  }
};

int64_t cells_of(const int32_t d[3]) { return (int64_t)d[0] * d[1] * d[2]; }

// Reads and checks the header; leaves the stream at the grid.  crc is updated over it.
int read_header(FILE* f, dmf_grid_header* h, uint32_t* crc) {
  uint8_t buf[kHeaderBytes];
  if (fread(buf, 1, kHeaderBytes, f) != kHeaderBytes) return fail(DMF_ERR_INVALID, "grid file: short header");
  uint32_t ver, hb, resv;
  memcpy(&ver, buf + 8, 4);
  memcpy(&hb, buf + 12, 4);
  memcpy(&resv, buf + 28, 4);
  if (memcmp(buf, kMagic, 8) != 0) return fail(DMF_ERR_INVALID, "grid file: bad magic");
  if (ver != kVersion || hb != kHeaderBytes || resv != 0) return fail(DMF_ERR_INVALID, "grid file: unsupported version");
  memcpy(h->dims, buf + 16, 12);
  memcpy(h->bounds, buf + 32, 48);
  memcpy(&h->params, buf + 80, 24);
  for (int a = 0; a < 3; ++a)
    if (h->dims[a] < 1 || h->dims[a] > (1 << 20)) return fail(DMF_ERR_INVALID, "grid file: bad dims");
  *crc = crc32().update(0, buf, kHeaderBytes);
  return DMF_OK;
}

}  // namespace
}  // namespace dmf

using namespace dmf;

extern "C" {

int dmf_grid_save(const char* path, const dmf_grid_header* h, const int16_t* logodds) {
  DMF_API_BEGIN
  if (!path || !h || !logodds) return fail(DMF_ERR_INVALID, "null argument");
  for (int a = 0; a < 3; ++a)
    if (h->dims[a] < 1 || h->dims[a] > (1 << 20)) return fail(DMF_ERR_INVALID, "bad dims");
  uint8_t head[kHeaderBytes];
  put_header(h, head);
  // written to a unique temporary file in the target's directory (mkstemp: two writers of one
  // path never share it), flushed to disk, renamed over path, then the directory itself is
  // synced so that the new entry survives a crash: a crash or a full disk mid-write leaves the
  // previous file intact
  std::string tmp = std::string(path) + ".XXXXXX";
  const int fd = mkstemp(&tmp[0]);
  if (fd < 0) return fail(DMF_ERR_INVALID, "cannot create a temporary file beside %s", path);
  // mkstemp creates the file 0600; give it the mode a plain fopen would have (0666 less the
  // umask), or the mode of the file it replaces
  {
    struct stat st;
    mode_t mode;
    if (stat(path, &st) == 0) {
      mode = st.st_mode & 07777;
    } else {
      const mode_t um = umask(0);
      umask(um);
      mode = 0666 & ~um;
    }
    if (fchmod(fd, mode) != 0) {
      close(fd);
      unlink(tmp.c_str());
      return fail(DMF_ERR_INVALID, "cannot set the mode of %s", tmp.c_str());
    }
  }
  File out;
  out.f = fdopen(fd, "wb");
  if (!out.f) {
    close(fd);
    unlink(tmp.c_str());
    return fail(DMF_ERR_INVALID, "cannot open %s for writing", tmp.c_str());
  }
  const size_t n = (size_t)cells_of(h->dims);
  uint32_t crc = crc32().update(0, head, sizeof(head));
  crc = crc32().update(crc, logodds, n * sizeof(int16_t));
  const bool ok = fwrite(head, 1, sizeof(head), out.f) == sizeof(head) &&
                  fwrite(logodds, sizeof(int16_t), n, out.f) == n && fwrite(&crc, 4, 1, out.f) == 1 &&
                  fflush(out.f) == 0 && fsync(fileno(out.f)) == 0;
  const bool closed = fclose(out.f) == 0;
  out.f = nullptr;
  if (!ok || !closed) {
    unlink(tmp.c_str());
    return fail(DMF_ERR_INVALID, "short write to %s", tmp.c_str());
  }
  if (rename(tmp.c_str(), path) != 0) {
    unlink(tmp.c_str());
    return fail(DMF_ERR_INVALID, "cannot rename %s to %s", tmp.c_str(), path);
  }
  std::string dir(path);
  const size_t slash = dir.find_last_of('/');
  dir = slash == std::string::npos ? std::string(".") : (slash == 0 ? std::string("/") : dir.substr(0, slash));
  const int dfd = open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (dfd < 0) return fail(DMF_ERR_INVALID, "cannot open directory %s to sync it", dir.c_str());
  const bool synced = fsync(dfd) == 0;
  close(dfd);
  if (!synced) return fail(DMF_ERR_INVALID, "cannot sync directory %s", dir.c_str());
  return DMF_OK;
  DMF_API_END
}

int dmf_grid_load(const char* path, dmf_grid_header* h, int16_t* logodds, int64_t cap) {
  DMF_API_BEGIN
  if (!path || !h) return fail(DMF_ERR_INVALID, "null argument");
  File in;
  in.f = fopen(path, "rb");
  if (!in.f) return fail(DMF_ERR_INVALID, "cannot open %s", path);
  uint32_t crc = 0;
  DMF_TRY(read_header(in.f, h, &crc));
  const int64_t n = cells_of(h->dims);
  // the file's size must be exactly header + grid + checksum BEFORE a caller sizes a buffer
  // from the (not yet checksummed) dims
  struct stat sb;
  if (fstat(fileno(in.f), &sb) != 0 || (int64_t)sb.st_size != (int64_t)kHeaderBytes + 2 * n + 4)
    return fail(DMF_ERR_INVALID, "grid file: size does not match its dims");
  if (!logodds) return DMF_OK;  // header only
  if (cap < n) return fail(DMF_ERR_CAPACITY, "grid of %lld cells, buffer of %lld", (long long)n, (long long)cap);
  if (fread(logodds, sizeof(int16_t), (size_t)n, in.f) != (size_t)n) return fail(DMF_ERR_INVALID, "grid file: short grid");
  uint32_t stored = 0;
  if (fread(&stored, 4, 1, in.f) != 1) return fail(DMF_ERR_INVALID, "grid file: missing checksum");
  crc = crc32().update(crc, logodds, (size_t)n * sizeof(int16_t));
  if (crc != stored) return fail(DMF_ERR_INVALID, "grid file: checksum mismatch");
  if (fgetc(in.f) != EOF) return fail(DMF_ERR_INVALID, "grid file: trailing bytes");
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
