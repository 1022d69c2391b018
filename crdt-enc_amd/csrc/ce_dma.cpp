// ce_dma.cpp -- device -> host copies on the GPU's SDMA engines through the HSA runtime.
//
// A compaction's sealed file (tens of MB) goes down while the next batch runs on the device.  A
// copy the HIP runtime runs as a blit kernel writes host memory from the compute units, and every
// kernel beside it slows down several-fold for its whole duration (profiles/r04_c3_step.txt); an
// SDMA engine leaves the compute units and their memory path alone (tools/ubench_d2h_interference.hip).
// The HIP runtime in a torch process picks the blit for these copies, so the copy is issued to
// the engine directly: hsa_amd_memory_async_copy_on_engine with a completion signal.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "ce_internal.h"

namespace ce {

namespace {

struct AgentSearch {
  uint32_t domain = 0, bdf = 0;
  hsa_agent_t gpu{0}, cpu{0};
  bool gpu_found = false, cpu_found = false;
};

hsa_status_t visit_agent(hsa_agent_t a, void* p) {
  auto* s = static_cast<AgentSearch*>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !s->cpu_found) {
    s->cpu = a;
    s->cpu_found = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !s->gpu_found) {
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) == HSA_STATUS_SUCCESS &&
        hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom) == HSA_STATUS_SUCCESS &&
        bdf == s->bdf && dom == s->domain) {
      s->gpu = a;
      s->gpu_found = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

}  // namespace

bool dma_init(int device, DmaD2H* out) {
  *out = DmaD2H{};
  if (getenv("CE_DMA_OFF")) return false;
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  AgentSearch s;
  s.domain = (uint32_t)dom;
  s.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);  // function 0
  if (hsa_iterate_agents(visit_agent, &s) != HSA_STATUS_SUCCESS || !s.gpu_found || !s.cpu_found) return false;
  uint32_t mask = 0;
  if (hsa_amd_memory_copy_engine_status(s.cpu, s.gpu, &mask) != HSA_STATUS_SUCCESS) mask = 0;
  out->gpu = s.gpu;
  out->cpu = s.cpu;
  // the runtime's engine choice by default; CE_DMA_ENGINE=k: SDMA engine k when it is free
  out->engine = 0;
  if (const char* ev = getenv("CE_DMA_ENGINE")) {
    const int k = atoi(ev);
    if (k >= 0 && k < 32 && (mask & (1u << k))) out->engine = 1u << k;
  }
  out->ok = true;
  return true;
}

bool dma_d2h(const DmaD2H& d, void* dst, const void* src, size_t n, hsa_signal_t sig) {
  if (!d.ok) return false;
  hsa_signal_store_screlease(sig, 1);
  hsa_status_t st;
  if (d.engine)
    st = hsa_amd_memory_async_copy_on_engine(dst, d.cpu, src, d.gpu, n, 0, nullptr, sig,
                                             static_cast<hsa_amd_sdma_engine_id_t>(d.engine), true);
  else
    st = hsa_amd_memory_async_copy(dst, d.cpu, src, d.gpu, n, 0, nullptr, sig);
  if (st != HSA_STATUS_SUCCESS) {
    hsa_signal_store_screlease(sig, 0);
    return false;
  }
  return true;
}

void dma_wait(hsa_signal_t sig) {
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) != 0) {
  }
}

bool dma_signal(hsa_signal_t* sig) { return hsa_signal_create(0, 0, nullptr, sig) == HSA_STATUS_SUCCESS; }

void dma_signal_destroy(hsa_signal_t sig) {
  if (sig.handle) (void)hsa_signal_destroy(sig);
}

}  // namespace ce
