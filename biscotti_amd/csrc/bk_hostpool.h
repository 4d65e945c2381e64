// bk_hostpool.h -- host worker threads for the row-fed entry (bk_multikrum_rows).
//
// The verifier's batch arrives as n separately allocated host rows (Go's
// [][]float64 of DistSys/krum.go:100-166, one slice per peer's RPC).  Before
// the first byte can cross PCIe the rows must sit in pinned memory; one core
// copying 4.3 GB (config D) serially costs more than the whole PCIe transfer.
// The pool packs the rows into the pinned stage on several cores, item by
// item, while the calling thread hands each finished chunk to the copy engine.
#ifndef BK_HOSTPOOL_H_
#define BK_HOSTPOOL_H_

#include <emmintrin.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bk {

// A fixed set of worker threads running the numbered items of one job at a
// time.  The caller releases items progressively (release(k): items [0, k) may
// be taken, in order), may run items itself (help()), and ends the job with
// end(), which hands out nothing more and waits until no item is in flight --
// so the job function, which lives on the caller's stack, is no longer used.
class HostPool {
public:
    explicit HostPool(int workers) {
        for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            stop_flag_.store(true, std::memory_order_relaxed);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    HostPool(const HostPool &) = delete;
    HostPool &operator=(const HostPool &) = delete;

    int workers() const { return (int)th_.size(); }

    void begin(int nitems, const std::function<void(int)> *fn) {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = fn;
        n_ = nitems;
        next_ = released_ = inflight_ = 0;
        ticket_.fetch_add(1, std::memory_order_release);
    }
    void release(int upto) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (upto > n_) upto = n_;
            if (upto > released_) released_ = upto;
            ticket_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    // run one released item on the calling thread; false if none was waiting
    bool help() {
        int i;
        const std::function<void(int)> *f;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!job_ || next_ >= released_) return false;
            i = next_++;
            ++inflight_;
            f = job_;
        }
        (*f)(i);
        finish_one();
        return true;
    }
    void end() {
        std::unique_lock<std::mutex> lk(mu_);
        released_ = next_;  // nothing further is handed out
        done_.wait(lk, [&] { return inflight_ == 0; });
        job_ = nullptr;
    }

private:
    void finish_one() {
        std::lock_guard<std::mutex> lk(mu_);
        if (--inflight_ == 0) done_.notify_all();
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            if (!stop_ && !(job_ && next_ < released_)) {
                // spin a little before sleeping: the next release of this
                // job (the next chunk) or the next call's job usually comes
                // within microseconds, and a futex wake-up costs tens of them
                const uint64_t seen = ticket_.load(std::memory_order_acquire);
                lk.unlock();
                for (int i = 0; i < kSpin && ticket_.load(std::memory_order_acquire) == seen &&
                                !stop_flag_.load(std::memory_order_relaxed);
                     ++i)
                    _mm_pause();
                lk.lock();
            }
            cv_.wait(lk, [&] { return stop_ || (job_ && next_ < released_); });
            if (stop_) return;
            const int i = next_++;
            ++inflight_;
            const std::function<void(int)> *f = job_;
            lk.unlock();
            (*f)(i);
            lk.lock();
            if (--inflight_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int n_ = 0, next_ = 0, released_ = 0, inflight_ = 0;
    bool stop_ = false;
    // bumped by every begin() / release(): what a spinning worker watches
    std::atomic<uint64_t> ticket_{0};
    std::atomic<bool> stop_flag_{false};
    // ~4k pauses: tens of microseconds (a spinning worker burns the
    // process's CPU share, which the caller and the copy engine's driver
    // thread also need)
    static constexpr int kSpin = 4000;
};

// Copy into pinned staging with non-temporal 16-B stores: the destination is
// read next by the copy engine, not by this core, so the stores bypass the
// cache (no read-for-ownership of the destination lines).  The caller issues
// _mm_sfence() before publishing that the bytes are in place.
inline void copy_to_stage(void *dst, const void *src, size_t bytes, bool nt = true) {
    if (!nt) {
        memcpy(dst, src, bytes);
        return;
    }
    char *d = (char *)dst;
    const char *s = (const char *)src;
    size_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (head > bytes) head = bytes;
    if (head) {
        memcpy(d, s, head);
        d += head;
        s += head;
        bytes -= head;
    }
    const size_t n64 = bytes / 64;
    for (size_t i = 0; i < n64; ++i) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(s + 0));
        const __m128i b = _mm_loadu_si128((const __m128i *)(s + 16));
        const __m128i c = _mm_loadu_si128((const __m128i *)(s + 32));
        const __m128i e = _mm_loadu_si128((const __m128i *)(s + 48));
        _mm_stream_si128((__m128i *)(d + 0), a);
        _mm_stream_si128((__m128i *)(d + 16), b);
        _mm_stream_si128((__m128i *)(d + 32), c);
        _mm_stream_si128((__m128i *)(d + 48), e);
        d += 64;
        s += 64;
    }
    const size_t rem = bytes - n64 * 64;
    if (rem) memcpy(d, s, rem);
}

}  // namespace bk

#endif  // BK_HOSTPOOL_H_
