// fp16 build of the fused LeNet conv stack (entry points suffixed _h); see lenet_conv.hip.
#define RK_LENET_H 1
#include "lenet_conv.hip"
