// native/ext/workqueue.hpp — the rate-limited exclusive-key work queue (client-go workqueue semantics).
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

// ----------------------------------------------------------------------------- work queue
class RateLimitingQueue {
  public:
    RateLimitingQueue(double base_delay, double max_delay, double qps, int burst)
        : base_(base_delay), max_(max_delay), qps_(qps), burst_(burst), tokens_(static_cast<double>(burst)) {}

    // Type
    bool add(const std::string& key) {
        std::lock_guard<std::mutex> g(mu_);
        return add_locked(key);
    }

    py::object try_get() {
        std::string key;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (queue_.empty()) return py::none();
            key = std::move(queue_.front());
            queue_.pop_front();
            processing_.insert(key);
            dirty_.erase(key);
        }
        return py::str(key);
    }

    bool done(const std::string& key) {
        std::lock_guard<std::mutex> g(mu_);
        processing_.erase(key);
        if (dirty_.count(key)) {
            queue_.push_back(key);
            return true;
        }
        return false;
    }

    size_t length() {
        std::lock_guard<std::mutex> g(mu_);
        return queue_.size();
    }
    size_t processing() {
        std::lock_guard<std::mutex> g(mu_);
        return processing_.size();
    }
    void shutdown() {
        std::lock_guard<std::mutex> g(mu_);
        shutting_down_ = true;
    }
    bool shutting_down() {
        std::lock_guard<std::mutex> g(mu_);
        return shutting_down_;
    }

    // Delaying
    bool add_after(const std::string& key, double delay, double now) {
        std::lock_guard<std::mutex> g(mu_);
        return add_after_locked(key, delay, now);
    }

    size_t promote(double now) {
        std::lock_guard<std::mutex> g(mu_);
        size_t n = 0;
        while (!heap_.empty() && heap_.top().ready <= now) {
            Waiting w = heap_.top();
            heap_.pop();
            auto it = waiting_ready_.find(w.key);
            if (it == waiting_ready_.end() || it->second != w.ready) continue;  // superseded
            waiting_ready_.erase(it);
            if (add_locked(w.key)) ++n;
        }
        return n;
    }

    double next_ready_in(double now) {
        std::lock_guard<std::mutex> g(mu_);
        while (!heap_.empty()) {
            const Waiting& w = heap_.top();
            auto it = waiting_ready_.find(w.key);
            if (it != waiting_ready_.end() && it->second == w.ready) break;
            heap_.pop();
        }
        if (heap_.empty()) return -1.0;
        return std::max(0.0, heap_.top().ready - now);
    }

    size_t waiting() {
        std::lock_guard<std::mutex> g(mu_);
        return waiting_ready_.size();
    }

    // Queued, being processed or waiting for a delayed add: a worker pass for the key is pending or running.
    bool busy(const std::string& key) {
        std::lock_guard<std::mutex> g(mu_);
        return dirty_.count(key) || processing_.count(key) || waiting_ready_.count(key);
    }

    // RateLimiting: MaxOf(ItemExponentialFailure(base, max), Bucket(qps, burst))
    double add_rate_limited(const std::string& key, double now) {
        std::lock_guard<std::mutex> g(mu_);
        double d = std::max(exp_when(key), bucket_when(now));
        add_after_locked(key, d, now);
        return d;
    }

    void forget(const std::string& key) {
        std::lock_guard<std::mutex> g(mu_);
        failures_.erase(key);
    }

    int num_requeues(const std::string& key) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = failures_.find(key);
        return it == failures_.end() ? 0 : it->second;
    }

  private:
    struct Waiting {
        double ready;
        uint64_t seq;
        std::string key;
    };
    struct Later {
        bool operator()(const Waiting& a, const Waiting& b) const {
            return a.ready != b.ready ? a.ready > b.ready : a.seq > b.seq;
        }
    };

    bool add_locked(const std::string& key) {
        if (shutting_down_ || dirty_.count(key)) return false;
        dirty_.insert(key);
        if (processing_.count(key)) return false;
        queue_.push_back(key);
        return true;
    }

    bool add_after_locked(const std::string& key, double delay, double now) {
        if (shutting_down_) return false;
        if (delay <= 0) return add_locked(key);
        double ready = now + delay;
        auto it = waiting_ready_.find(key);
        if (it != waiting_ready_.end() && it->second <= ready) return false;
        waiting_ready_[key] = ready;
        heap_.push(Waiting{ready, ++seq_, key});
        return false;
    }

    double exp_when(const std::string& key) {
        int& f = failures_[key];
        int e = f++;
        if (e >= 64) return max_;
        double d = base_ * std::ldexp(1.0, e);
        return d > max_ ? max_ : d;
    }

    double bucket_when(double now) {
        if (qps_ <= 0) return 0.0;
        if (!has_last_) {
            last_ = now;
            has_last_ = true;
        }
        double elapsed = now - last_;
        if (elapsed > 0) {
            tokens_ = std::min(static_cast<double>(burst_), tokens_ + elapsed * qps_);
            last_ = now;
        }
        tokens_ -= 1.0;
        return tokens_ >= 0 ? 0.0 : -tokens_ / qps_;
    }

    std::mutex mu_;
    double base_, max_, qps_;
    int burst_;
    double tokens_;
    double last_ = 0.0;
    bool has_last_ = false;
    std::unordered_map<std::string, int> failures_;
    std::deque<std::string> queue_;
    std::unordered_set<std::string> dirty_, processing_;
    std::priority_queue<Waiting, std::vector<Waiting>, Later> heap_;
    std::unordered_map<std::string, double> waiting_ready_;
    uint64_t seq_ = 0;
    bool shutting_down_ = false;
};
