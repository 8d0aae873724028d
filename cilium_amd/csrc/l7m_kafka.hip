#include "l7m_device.h"
namespace l7m {
hipError_t launch_kafka(const uint32_t*, const KafkaHeader&, const uint8_t*, uint64_t, const uint64_t*,
                        uint64_t, int32_t*, unsigned long long*, hipStream_t, int) {
  return hipErrorInvalidValue;
}
}  // namespace l7m
