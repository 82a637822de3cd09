/*
 * batch_reduce_entry.hpp — a new schedule entry for oneCCL's src/sched/entry
 * (integration/0004-nreduce-fused-fanin.patch).
 *
 * nreduce's reduce-scatter (src/coll/algorithms/allreduce/allreduce.cpp:376-394)
 * folds each peer's chunk into reduce_buf with its own recv_reduce_entry: P-1
 * chained 2-input reduces, 3(P-1) chunk-sizes of memory traffic.  With the
 * peers' chunks received into their slots of the schedule's tmp buffer, this
 * entry folds all of them in one ccl_comp_batch_reduce request (one K-input
 * kernel on the GPU, one pass on the CPU path): P+1 chunk-sizes.
 *
 *   inout = op(in + offsets[K-1], ... op(in + offsets[1], inout))
 *
 * offsets are in elements from in_buf; offsets[0] names the accumulator's
 * slot and is not read (src/comp/comp.cpp:216-245).  The request is started
 * in start() and polled in update(), like reduce_local_entry's device path
 * (reduce_local_entry.cpp:116-131), so the worker progresses other entries
 * meanwhile -- when the entry is a barrier (sched->add_barrier() after it, as
 * 0004 does), the only case in which the progress loop holds back the entries
 * that read its result (sched.cpp:485).  Otherwise it completes in start().
 * C++11, as the rest of src/ (CMakeLists.txt:172).
 */
#pragma once

#include "common/global/global.hpp"
#include "comp/comp.hpp"
#include "sched/entry/entry.hpp"
#include "sched/queue/queue.hpp"

#include "mi_ccl_comp_async.hpp"

#include <algorithm>
#include <utility>
#include <vector>

class batch_reduce_entry final : public sched_entry {
public:
    static constexpr const char* class_name() noexcept {
        return "BATCH_REDUCE";
    }

    batch_reduce_entry() = delete;
    batch_reduce_entry(const batch_reduce_entry& other) = delete;
    batch_reduce_entry& operator=(const batch_reduce_entry& other) = delete;
    batch_reduce_entry(ccl_sched* sched,
                       ccl_buffer in_buf,
                       std::vector<size_t> offsets,
                       size_t cnt,
                       ccl_buffer inout_buf,
                       const ccl_datatype& dtype,
                       ccl::reduction reduction_op)
            : sched_entry(sched),
              in_buf(in_buf),
              offsets(std::move(offsets)),
              cnt(cnt),
              inout_buf(inout_buf),
              dtype(dtype),
              op(reduction_op),
              fn(sched->coll_attr.reduction_fn) {
        CCL_THROW_IF_NOT(op != ccl::reduction::custom || fn,
                         "custom reduction requires user provided callback",
                         ", op ",
                         ccl_reduction_to_str(op),
                         ", fn ",
                         fn);
        CCL_THROW_IF_NOT(!this->offsets.empty(), "batch reduce needs the accumulator's slot");
    }

    ~batch_reduce_entry() override {
        if (req) {  // the schedule is torn down mid-flight: the GPU must be done with both buffers
            ccl_comp_request_wait(req);
            ccl_comp_request_free(req);
        }
    }

    void start() override {
        const size_t bytes = cnt * dtype.size();
        const size_t in_bytes =
            (*std::max_element(offsets.begin(), offsets.end()) + cnt) * dtype.size();
        const ccl::fn_context context = { sched->coll_attr.match_id.c_str(),
                                          inout_buf.get_offset() };
        ccl_comp_batch_reduce_start(sched, /* host memory unless its collective has a stream */
                                    in_buf.get_ptr(in_bytes),
                                    offsets,
                                    cnt,
                                    inout_buf.get_ptr(bytes),
                                    nullptr, /* out_count */
                                    dtype,
                                    op,
                                    fn,
                                    &context,
                                    0, /* bf16_keep_precision_mode */
                                    &req);
        if (!is_barrier()) {
            // only a barrier entry holds back the entries after it
            // (sched.cpp:485): without one, finish here (0004 adds one)
            ccl_comp_request_wait(req);
            ccl_comp_request_free(req);
            req = nullptr;
            status = ccl_sched_entry_status_complete;
            return;
        }
        status = ccl_sched_entry_status_started;
        update();
    }

    void update() override {
        if (req && ccl_comp_request_test(req)) {
            ccl_comp_request_free(req);
            req = nullptr;
            status = ccl_sched_entry_status_complete;
        }
    }

    const char* name() const override {
        return class_name();
    }

protected:
    void dump_detail(std::stringstream& str) const override {
        ccl_logger::format(str,
                           "dt ",
                           ccl::global_data::get().dtypes->name(dtype),
                           ", in_buf ",
                           in_buf,
                           ", inputs ",
                           offsets.size(),
                           ", cnt ",
                           cnt,
                           ", inout_buf ",
                           inout_buf,
                           ", op ",
                           ccl_reduction_to_str(op),
                           ", red_fn ",
                           fn,
                           "\n");
    }

private:
    ccl_buffer in_buf;
    std::vector<size_t> offsets;
    size_t cnt;
    ccl_buffer inout_buf;
    ccl_datatype dtype;
    ccl::reduction op;
    ccl::reduction_fn fn;
    ccl_comp_request* req = nullptr;
};
