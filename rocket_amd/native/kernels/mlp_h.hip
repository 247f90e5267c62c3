// fp16 build of the fused LeNet classifier / weight-gradient kernels (entry points suffixed _h); see mlp.hip.
#define RK_LENET_H 1
#include "mlp.hip"
