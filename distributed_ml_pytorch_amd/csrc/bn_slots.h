#pragma once
// Shared by the device code and the host bindings.
namespace dmp {
// BatchNorm statistics travel as [2][kBnSlots][C] fp32 slot sums: producers
// (conv epilogues, the BN reduction pass) atomically add their per-block sums
// into slot blockIdx % kBnSlots, the finalize kernel reads kBnSlots rows per
// channel instead of one per producer block (thousands) and zeroes the slots
// for their next use (they are persistent per layer).
constexpr int kBnSlots = 64;
// a slot buffer is [2][kBnSlots][C] fp32 followed by kBnTail words: word 0 is
// the arrival ticket of the single-pass reduce + finalize (bn.hip)
constexpr int kBnTail = 4;
}  // namespace dmp
