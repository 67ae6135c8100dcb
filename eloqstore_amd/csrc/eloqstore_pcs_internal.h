// eloqstore_pcs_internal.h — launch entry points shared by the C ABI
// (pcs_capi.cpp) and the kernels (pcs_kernels.hip).  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pcs {

// mode: 0 digest, 1 validate, 2 stamp.  algo: 0 XXH3-64, 1 XXH64.
// Fixed-stride pages, any shape (odd shapes run as a descriptor batch built
// on the device).
hipError_t run_pages(int mode, int algo, const uint8_t* pages, uint64_t page_size, uint64_t n, uint64_t* out,
                     uint8_t* ok, unsigned long long* first_bad, hipStream_t s);

// Descriptor batch: range i = [base + off[i], +len[i]).  skip = 8 applies the
// page convention (digest over [8, len), stored digest at [0, 8)); skip = 0
// hashes the raw range.  seed is used by XXH64 only (XXH3 path is seed 0).
hipError_t run_desc(int mode, int algo, const uint8_t* base, const uint64_t* off, const uint32_t* len, uint64_t n,
                    int skip, uint64_t seed, uint64_t* out, uint8_t* ok, unsigned long long* first_bad,
                    hipStream_t s);

// Page list: page i is the absolute device-visible address ptrs[i] (pool
// pages in registered host memory), all of size page_size.  ptrs, out and ok
// may live in pinned host memory.  No first_bad word: the caller scans the
// verdicts.  Only the fast shapes (list_shape_ok) are supported.
inline bool list_shape_ok(int algo, uint64_t P) {
    return algo == 0 ? (P % 256 == 0 && P >= 256 && P <= 0xFFFFFFFFull)
                     : (P % 64 == 0 && P >= 128 && P <= 0xFFFFFFFFull);
}
// host_ptrs, if given, is a host-readable copy of the list: small batches
// pass it in the kernel arguments instead.
hipError_t run_list(int mode, int algo, const uint64_t* ptrs, const uint64_t* host_ptrs, uint64_t page_size,
                    uint64_t n, uint64_t* out, uint8_t* ok, hipStream_t s);

hipError_t run_gen_pages(uint8_t* pages, uint64_t page_size, uint64_t n, uint64_t seed, uint64_t first_page,
                         hipStream_t s);
hipError_t run_gen_desc(uint8_t* base, const uint64_t* off, const uint32_t* len, uint64_t n, uint64_t seed,
                        uint64_t first_page, hipStream_t s);
hipError_t run_flip(uint8_t* pages, uint64_t page_size, uint64_t n, uint64_t every, uint64_t byte_off,
                    hipStream_t s);
// ManifestBuilder::CalcChecksum over a device-resident content buffer
hipError_t run_manifest(const uint8_t* content, uint64_t len, uint64_t* out, hipStream_t s);
// Event-fenced device scratch (see ScratchPool in pcs_kernels.hip): the
// buffer is reused only after the work queued on `s` at release completes.
hipError_t scratch_acquire(size_t bytes, void** out, int* id);
hipError_t scratch_release(int id, hipStream_t s);
int set_tuning(int key, int64_t value);
// Decrements a positive knob by one and returns true (PCS_TUNE_FAIL_INJECT).
bool take_tuning(int key);
int64_t get_tuning(int key);
// Plain streaming read of [buf, buf + bytes) (the HBM read ceiling): one
// folded word per 4 KiB page into out[0 .. ceil(bytes / 4096)).
hipError_t run_stream_read(const uint8_t* buf, uint64_t bytes, uint64_t* out, hipStream_t s);

// Pre-armed validate service (pcs_service_*): a mailbox in pinned host
// memory, read by the waiting kernel through its device alias.  It holds up
// to kServiceMaxLines request lines, one per concurrent caller; line k is
// served by workgroups [k * wpl, (k + 1) * wpl) of the kernel.  The first
// kServiceLineWords words of a line (two 64-byte lines) carry a whole small
// request: seq = generation << 32 | count, page count, page size, a check
// word and the first kServiceLinePtrs page addresses, so the poll that sees a
// new seq brings in a request of up to 12 pages.  The host writes seq last.
// The 16 words arrive as separate per-lane loads, so nothing makes them one
// snapshot: the check word (the sum of service_word_mix over the other 15
// words, written by the host just before seq) is what proves that a poll saw
// one request's words and not a new seq beside an older request's page
// addresses.  A poll whose words do not add up to their check word is
// ignored and the line is read again.  Verdicts are 32-bit words stored
// system-scope.  `gen` names the newest generation: a kernel of an older one
// leaves at its next poll.
constexpr int kServiceMaxPages = 256;
constexpr int kServiceMaxLines = 8;
constexpr int kServiceLineWords = 16;
constexpr int kServiceCheckWord = 3;
constexpr int kServiceLinePtrs = kServiceLineWords - 4;
constexpr uint32_t kServicePending = 0xA5A5A5A5u;
constexpr uint64_t kServiceStamp = 1ull << 32;  // in the page-size word: a stamp request
struct ServiceLine {
    alignas(64) uint64_t seq;
    uint64_t n;
    uint64_t page_size;               // | kServiceStamp for a stamp request
    uint64_t check;                   // sum of service_word_mix(word i, i) over the other line words
    uint64_t ptrs[kServiceMaxPages];  // device-visible page addresses
    alignas(64) uint32_t ok[kServiceMaxPages];
    alignas(64) uint64_t torn_seq;    // kernel: the last seq it saw beside words that failed the check
};
constexpr int kServiceMaxWorkgroups = 256;  // lines * workgroups per line
struct ServiceBox {
    alignas(64) uint64_t stop;  // host: 1 ends every waiting kernel
    uint64_t gen;               // host: the newest generation (written before its kernel is queued)
    ServiceLine line[kServiceMaxLines];
    // kernel: departed[w] = the generation of the last workgroup w to leave,
    // stored after every verdict / header store of it is visible system-wide
    alignas(64) uint32_t departed[kServiceMaxWorkgroups];
};
static_assert(offsetof(ServiceLine, ptrs) == 4 * sizeof(uint64_t), "line words: seq, n, page_size, check, ptrs");
static_assert(offsetof(ServiceBox, gen) == offsetof(ServiceBox, stop) + 8, "stop and gen are one poll's two words");
// murmur3's 64-bit finaliser over (word, position): a word read from an older
// request changes the sum by a pseudo-random 64-bit amount.
__host__ __device__ inline uint64_t service_word_mix(uint64_t w, uint64_t i) {
    uint64_t x = w ^ (i * 0x9E3779B97F4A7C15ull) ^ 0xD6E8FEB86659FD93ull;
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}
// Queue one service kernel of generation `gen`: lines * wpl workgroups,
// workgroup w serving line w / wpl.  Each serves its line's requests of that
// generation until idle_ticks pass without one or, between requests, it has
// lived life_ticks (both on the 100 MHz real-time clock), or stop is set, or
// the box names a newer generation; then it stores gen into departed[w].
// exit_ticks: test only (a kernel that serves nothing and leaves that many
// ticks late; 0 in production).
hipError_t run_service(ServiceBox* d_box, int lines, int wpl, uint32_t gen, uint64_t idle_ticks, uint64_t life_ticks,
                       uint64_t exit_ticks, hipStream_t s);

}  // namespace pcs
