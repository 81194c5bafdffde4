// Instantiates the reduce, fused-allreduce and pipelined-allreduce kernels of one op
// (-DCOLL_OP=<OMPI_AMD_OP_*>) for every type op/base defines it on, and
// exports that op's launch rows (coll_kernels.h).  One object per op keeps
// the template instantiations in parallel compile jobs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <utility>

#include "coll_kernels.h"

#ifndef COLL_OP
#error "build with -DCOLL_OP=<op index>"
#endif

namespace ompi_amd {
namespace {

template <int OP, int TYPE>
hipError_t red_launch_slot(dim3 grid, const ptr_set &src, const ptr_set &dst, int ndst, int n,
                           int order, int flags, const red_jobs &jobs, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        if (n <= 8)
            hipLaunchKernelGGL((reduce_kernel<T, OP, 8>), grid, dim3(kXferThreads), 0, s, src, dst,
                               ndst, n, order, flags, jobs);
        else
            hipLaunchKernelGGL((reduce_kernel<T, OP, kMaxRanks>), grid, dim3(kXferThreads), 0, s,
                               src, dst, ndst, n, order, flags, jobs);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int OP, int TYPE>
hipError_t fused_launch_slot(dim3 grid, const fused_args &a, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        hipLaunchKernelGGL((fused_allreduce_kernel<T, OP>), grid, dim3(kXferThreads), 0, s, a);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int OP, int TYPE>
hipError_t pipe_launch_slot(unsigned groups, const pipe_args &a, hipStream_t s) {
    if constexpr (slot_supported(OP, TYPE)) {
        using T = typename type_of<TYPE>::type;
        if (a.n > 8) return hipErrorInvalidValue;  // the host runs the phased schemes there
        // Workgroup w waits for workgroup w of every peer, so every
        // colocated rank's grid must be resident at once: at most half the
        // GPU's capacity for this kernel over the ranks sharing it (half:
        // a second communicator's pipelined call may run beside it).  The
        // same on every rank (same kernel, same GPU model, agreed colocated).
        static const int64_t cap = [] {
            int per_cu = 0, cus = 0, dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &per_cu, reinterpret_cast<const void *>(&pipe_allreduce_kernel<T, OP, 8>),
                    kXferThreads, 0) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
                (void)hipGetLastError();
                return (int64_t)64;
            }
            return std::max<int64_t>(1, (int64_t)per_cu * cus / 2);
        }();
        const int64_t fit = std::max<int64_t>(1, cap / std::max(1, a.colocated));
        const dim3 g((unsigned)std::min<int64_t>(groups, fit)), b(kXferThreads);
        hipLaunchKernelGGL((pipe_allreduce_kernel<T, OP, 8>), g, b, 0, s, a);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}

template <int OP, int... T>
constexpr std::array<red_launch_fn, OMPI_AMD_TYPE_COUNT> make_red_row(std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &red_launch_slot<OP, T> : (red_launch_fn) nullptr)...}};
}
template <int OP, int... T>
constexpr std::array<fused_launch_fn, OMPI_AMD_TYPE_COUNT> make_fused_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &fused_launch_slot<OP, T> : (fused_launch_fn) nullptr)...}};
}

template <int OP, int... T>
constexpr std::array<pipe_launch_fn, OMPI_AMD_TYPE_COUNT> make_pipe_row(
    std::integer_sequence<int, T...>) {
    return {{(slot_supported(OP, T) ? &pipe_launch_slot<OP, T> : (pipe_launch_fn) nullptr)...}};
}

const auto g_red_row = make_red_row<COLL_OP>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{});
const auto g_fused_row = make_fused_row<COLL_OP>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{});
const auto g_pipe_row = make_pipe_row<COLL_OP>(std::make_integer_sequence<int, OMPI_AMD_TYPE_COUNT>{});

}  // namespace

#define ROW_NAME2(a, b) a##b
#define ROW_NAME(a, b) ROW_NAME2(a, b)
const red_launch_fn *ROW_NAME(red_row_, COLL_OP)() { return g_red_row.data(); }
const fused_launch_fn *ROW_NAME(fused_row_, COLL_OP)() { return g_fused_row.data(); }
const pipe_launch_fn *ROW_NAME(pipe_row_, COLL_OP)() { return g_pipe_row.data(); }

}  // namespace ompi_amd
