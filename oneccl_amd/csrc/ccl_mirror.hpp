// ccl_mirror.hpp — standalone mirror of the oneCCL types that cross the
// src/comp boundary.  Used only when comp.cpp is built OUTSIDE the oneCCL
// tree (tests, bench, this repo).  Inside the tree (-DMI_ONECCL_TREE) the
// real headers are included instead; the declarations below reproduce their
// names, namespaces (ccl::v1) and enumerator values so the exported
// symbols mangle identically:
//   ccl::reduction, ccl::datatype       include/oneapi/ccl/types.hpp:41-69
//   ccl::fn_context, ccl::reduction_fn  include/oneapi/ccl/types.hpp:117-124
//   ccl::status                         src/internal_types.hpp:29-37
//   ccl_datatype                        src/common/datatype/datatype.hpp:31-54
//   ccl_bf16_impl_type                  src/comp/bf16/bf16_utils.hpp:26
//   ccl_fp16_impl_type                  src/comp/fp16/fp16_utils.hpp:26-32
//   ccl::exception                      include/oneapi/ccl/exception.hpp
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

namespace ccl {
namespace v1 {

enum class reduction : int { sum = 0, prod, min, max, custom };

enum class datatype : int {
    int8 = 0,
    uint8,
    int16,
    uint16,
    int32,
    uint32,
    int64,
    uint64,
    float16,
    float32,
    float64,
    bfloat16,
};

typedef struct {
    const char* match_id;
    const size_t offset;
} fn_context;

typedef void (*reduction_fn)(const void*, size_t, void*, size_t*, ccl::v1::datatype,
                             const ccl::v1::fn_context*);

class exception : public std::exception {
public:
    explicit exception(const std::string& info) : msg(std::string("oneCCL: ") + info) {}
    const char* what() const noexcept override { return msg.c_str(); }

private:
    std::string msg;
};

}  // namespace v1
using namespace v1;

enum status : int {
    success = 0,
    out_of_resource,
    invalid_arguments,
    runtime_error,
    blocked_due_to_resize,
    last_value
};

}  // namespace ccl

// The one thing src/comp reads of a schedule: its collective's stream
// (sched->coll_param.stream, src/sched/sched_base.hpp:151,
// src/coll/coll_param.hpp:129; the reference's comp.cpp:137).  The
// standalone ccl_sched carries only that; the mangled names depend on the
// class name alone.
class ccl_stream;  // opaque
struct ccl_coll_param {
    ccl_stream* stream = nullptr;
};
class ccl_sched {
public:
    ccl_coll_param coll_param;
};

class ccl_datatype {
public:
    ccl_datatype() = default;
    ccl_datatype(ccl::datatype idx, size_t size) : m_idx(idx), m_size(size) {}
    ccl::datatype idx() const noexcept { return m_idx; }
    size_t size() const {
        if (m_size == 0) throw ccl::exception("non-positive datatype size 0");
        return m_size;
    }

private:
    ccl::datatype m_idx = ccl::datatype::int8;
    size_t m_size = sizeof(int8_t);
};

typedef enum { ccl_bf16_scalar = 0, ccl_bf16_avx512f, ccl_bf16_avx512bf } ccl_bf16_impl_type;

typedef enum {
    ccl_fp16_no_compiler_support = 0,
    ccl_fp16_no_hardware_support,
    ccl_fp16_f16c,
    ccl_fp16_avx512f,
    ccl_fp16_avx512fp16
} ccl_fp16_impl_type;

extern std::map<ccl_bf16_impl_type, std::string> bf16_impl_names;
extern std::map<ccl_fp16_impl_type, std::string> fp16_impl_names;
extern std::map<ccl_fp16_impl_type, std::string> fp16_env_impl_names;

// src/comp/comp.hpp:23-51
ccl::status ccl_comp_copy(const void* in_buf, void* out_buf, size_t count, bool use_nontemporal = false);

ccl::status ccl_comp_reduce(ccl_sched* sched, const void* in_buf, size_t in_count, void* inout_buf,
                            size_t* out_count, const ccl_datatype& dtype, ccl::reduction reduction,
                            ccl::reduction_fn reduction_fn, const ccl::fn_context* context = nullptr);

ccl::status ccl_comp_batch_reduce(const void* in_buf, const std::vector<size_t>& offsets, size_t in_count,
                                  void* inout_buf, size_t* out_count, const ccl_datatype& dtype,
                                  ccl::reduction reduction, ccl::reduction_fn reduction_fn,
                                  const ccl::fn_context* context, int bf16_keep_precision_mode, float* tmp,
                                  float* acc);

const char* ccl_reduction_to_str(ccl::reduction type);

// src/comp/bf16/bf16.hpp:26-38, src/comp/fp16/fp16.hpp:21-35
void ccl_bf16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, ccl::reduction op);
void ccl_fp16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, ccl::reduction op);
void ccl_convert_fp32_to_bf16_arrays(void*, void*, size_t);
void ccl_convert_bf16_to_fp32_arrays(void*, float*, size_t);
void ccl_convert_fp32_to_bf16(const void* src, void* dst);  // 16 elements
void ccl_convert_bf16_to_fp32(const void* src, void* dst);  // 16 elements
void ccl_convert_fp32_to_fp16(const void* src, void* dst);  // 8 elements
void ccl_convert_fp16_to_fp32(const void* src, void* dst);  // 8 elements
