// TEST INFRASTRUCTURE ONLY. The CUDA execution model for ONE thread block, on CPU threads:
// prepended (g++ -include) to the reference kernel text tf_sampling_g.cu:105-170, which the
// Makefile pipes from /root/reference into g++ unchanged except for ONE added
// `__syncthreads();` after :165 (the write-after-read race on dists_i).
// Every `__shared__` array becomes a function-static object shared by the block's threads,
// `__syncthreads()` a std::barrier over blockDim.x threads, threadIdx a thread_local.
// The FPS oracle pin that does not depend on any GPU compiler.
#pragma once
#include <algorithm>
#include <barrier>
#include <memory>
#include <thread>
#include <vector>

namespace pn2emul {
struct dim3_ { int x = 0, y = 0, z = 0; };
inline thread_local dim3_ threadIdx_;
inline dim3_ blockIdx_, gridDim_, blockDim_;
inline std::barrier<>* bar_ = nullptr;
}  // namespace pn2emul

#define __global__
#define __shared__ static
#define __syncthreads() pn2emul::bar_->arrive_and_wait()
#define threadIdx pn2emul::threadIdx_
#define blockIdx pn2emul::blockIdx_
#define gridDim pn2emul::gridDim_
#define blockDim pn2emul::blockDim_
using std::min;
