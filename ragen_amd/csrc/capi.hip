// capi.hip — library-level helpers of the C ABI.
#include "common.hpp"

RMI_API const char* rmi_version(void) { return "ragen_amd 0.1.0 (gfx950)"; }

RMI_API int rmi_device_copy(void* dst, const void* src, size_t bytes, rmi_stream_t stream) {
  if ((!dst || !src) && bytes) return RMI_EINVAL;
  if (!bytes) return RMI_OK;
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, rmi::as_stream(stream)) == hipSuccess ? RMI_OK
                                                                                                    : RMI_EDEVICE;
}
