// TEST INFRASTRUCTURE ONLY (see fps_emul_head.h). Runs the kernel text as ONE block of
// `threads` CPU threads (gridDim.x = 1: the block loops over the b clouds, :113) against a
// caller workspace temp (n floats; the kernel indexes temp[blockIdx.x*n + k]).
extern "C" int pn2emul_fps(int b, int n, int m, int threads, const float* xyz, int* idx) {
  if (threads <= 0 || threads > 1024) return -22;
  std::vector<float> temp((size_t)(n > 0 ? n : 1));
  pn2emul::gridDim_ = {1, 1, 1};
  pn2emul::blockIdx_ = {0, 0, 0};
  pn2emul::blockDim_ = {threads, 1, 1};
  std::barrier<> bar(threads);
  pn2emul::bar_ = &bar;
  std::vector<std::thread> ts;
  ts.reserve(threads);
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([=, &temp] {
      pn2emul::threadIdx_ = {t, 0, 0};
      farthestpointsamplingKernel(b, n, m, xyz, temp.data(), idx);
    });
  for (auto& t : ts) t.join();
  pn2emul::bar_ = nullptr;
  return 0;
}
