// Optimizer hyperparameters for apply-on-arrival (asynchronous) parameter servers.
//
// A synchronous PS applies ONE optimizer step per round from the average of W pushes
// (reference: src/parameter_server.cpp:38-63 averages, :77-91 applies). An asynchronous PS applies
// every push on arrival, so one round is W optimizer steps. Run with the synchronous
// hyperparameters, that changes the optimizer, not just its noise:
//   * momentum decays W times per round (beta^W: 0.9 -> 0.43 at W = 8);
//   * Adam is invariant to the 1/W gradient scale, so W full-lr steps are taken per round (W x the
//     learning rate), and its bias corrections advance W times per round.
// The per-push hyperparameters below keep the per-ROUND behaviour of the synchronous optimizer
// (its EMA horizons, its steady-state displacement per round and its bias-correction schedule),
// and reduce to the synchronous ones exactly at W = 1:
//   SGD       grad x 1/W, lr, coupled weight decay wd/W    -> W pushes = one averaged step
//   momentum  grad x 1/W, beta_w = beta^(1/W), lr_w = lr (1 - beta_w) / (1 - beta), wd/W
//             (the buffer's steady state is the synchronous one, g / (1 - beta), and W pushes move
//             the weights by lr g / (1 - beta), the synchronous displacement per round)
//   Adam(W)   grad x 1, beta1_w = beta1^(1/W), beta2_w = beta2^(1/W), lr_w = lr / W, weight decay
//             unchanged (coupled: added to the unscaled gradient; AdamW: lr_w wd per push
//             compounds to ~lr wd per round). The bias corrections 1 - beta_w^t with t counted in
//             pushes equal 1 - beta^(t/W): the synchronous schedule counted in rounds.
#pragma once
#include <cmath>

namespace psd {

struct AsyncHyper {
  double lr_factor = 1.0;   // multiply the synchronous lr
  double grad_scale = 1.0;  // per-push gradient scale
  double momentum = 0.0;
  double beta1 = 0.9, beta2 = 0.999;
  double weight_decay = 0.0;
};

// kind: 0 SGD, 1 momentum, 2 Adam, 3 AdamW (OptimKind)
inline AsyncHyper async_hyper(int kind, int workers, double momentum, double beta1, double beta2,
                              double weight_decay) {
  AsyncHyper h;
  const double W = workers < 1 ? 1.0 : (double)workers;
  h.momentum = momentum;
  h.beta1 = beta1;
  h.beta2 = beta2;
  h.weight_decay = weight_decay;
  if (kind == 0) {
    h.grad_scale = 1.0 / W;
    h.weight_decay = weight_decay / W;
  } else if (kind == 1) {
    h.grad_scale = 1.0 / W;
    h.weight_decay = weight_decay / W;
    if (momentum > 0.0 && momentum < 1.0) {
      h.momentum = std::pow(momentum, 1.0 / W);
      h.lr_factor = (1.0 - h.momentum) / (1.0 - momentum);
    }
  } else {
    h.grad_scale = 1.0;
    h.lr_factor = 1.0 / W;
    h.beta1 = std::pow(beta1, 1.0 / W);
    h.beta2 = std::pow(beta2, 1.0 / W);
  }
  return h;
}

}  // namespace psd
