// timer.h -- kernel timers with the reference's TimerManager API, on hipEvents.
// Same classes and methods as detker/CUDA-Flash-Attention include/timer.h:11-164:
// TimerGPU records on the legacy default stream and Stop() synchronises
// (:50-64); TimerManager sums the intervals (:129-135).
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>

#include "error_utils.h"

class Timer {
public:
    virtual void Start() = 0;
    virtual void Stop() = 0;
    virtual float ElapsedMillis() = 0;
    virtual float ElapsedSeconds() { return ElapsedMillis() / 1000.0f; }
    virtual float TotalElapsedMillis() = 0;
    virtual float TotalElapsedSeconds() { return TotalElapsedMillis() / 1000.0f; }
    virtual void Reset() = 0;
    virtual ~Timer() = default;
};

class TimerGPU : public Timer {
    float total_ = 0.f, last_ = 0.f;
    bool running_ = false;
    hipEvent_t start_{}, stop_{};
    hipStream_t stream_ = nullptr;

public:
    explicit TimerGPU(hipStream_t stream = nullptr) : stream_(stream) {
        HIP_CHECK(hipEventCreate(&start_));
        HIP_CHECK(hipEventCreate(&stop_));
    }
    ~TimerGPU() override {
        (void)hipEventDestroy(start_);
        (void)hipEventDestroy(stop_);
    }
    void Start() override {
        if (running_) return;
        HIP_CHECK(hipEventRecord(start_, stream_));
        running_ = true;
    }
    void Stop() override {
        if (!running_) return;
        HIP_CHECK(hipEventRecord(stop_, stream_));
        HIP_CHECK(hipEventSynchronize(stop_));
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, start_, stop_));
        total_ += ms;
        last_ = ms;
        running_ = false;
    }
    float ElapsedMillis() override { return last_; }
    float TotalElapsedMillis() override { return total_; }
    void Reset() override { total_ = last_ = 0.f; running_ = false; }
};

class TimerCPU : public Timer {
    std::chrono::high_resolution_clock::time_point t0_;
    float total_ = 0.f, last_ = 0.f;
    bool running_ = false;

public:
    void Start() override {
        if (running_) return;
        t0_ = std::chrono::high_resolution_clock::now();
        running_ = true;
    }
    void Stop() override {
        if (!running_) return;
        last_ = std::chrono::duration<float, std::milli>(std::chrono::high_resolution_clock::now() - t0_).count();
        total_ += last_;
        running_ = false;
    }
    float ElapsedMillis() override { return last_; }
    float TotalElapsedMillis() override { return total_; }
    void Reset() override { total_ = last_ = 0.f; running_ = false; }
};

class TimerManager {
    Timer* timer_ = nullptr;
    float total_ = 0.f;

public:
    void Start() { timer_->Start(); }
    void Stop() {
        timer_->Stop();
        total_ += timer_->ElapsedMillis();
    }
    float ElapsedSecondsTimer() { return timer_->ElapsedSeconds(); }
    float ElapsedMillisTimer() { return timer_->ElapsedMillis(); }
    float TotalElapsedMillis() { return total_; }
    float TotalElapsedSeconds() { return total_ / 1000.0f; }
    float TotalElapsedSecondsTimer() { return timer_->TotalElapsedSeconds(); }
    float TotalElapsedMillisTimer() { return timer_->TotalElapsedMillis(); }
    void ResetTimer() { timer_->Reset(); }
    void Reset() { total_ = 0.f; }
    // extension: account device time measured elsewhere (the multi-GPU host API)
    void AddMillis(float ms) { total_ += ms; }
    void SetTimer(Timer* t) { timer_ = t; }
};
