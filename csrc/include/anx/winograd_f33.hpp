// Winograd F(3x3, 3x3), points {0, 1, -1, 2, inf} (Cook-Toom, exact rationals; B^T rows scaled to
// small integers, G rows scaled inversely: `tools/gen_winograd.py --m 3 --r 3 --pts 0,1,-1,2`).
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A   for a 5x5 input tile d and a 3x3 filter g.
// Used by Conv1 after its polyphase (stride -> channels) rewrite: hip/conv1_wino.hip.
#pragma once
namespace anx::wino33 {
constexpr int kM = 3, kR = 3, kN = 5;
constexpr float kAT[3][5] = {
    {1.0f, 1.0f, 1.0f, 1.0f, 0.0f},
    {0.0f, 1.0f, -1.0f, 2.0f, 0.0f},
    {0.0f, 1.0f, 1.0f, 4.0f, 1.0f}};

constexpr float kBT[5][5] = {
    {2.0f, -1.0f, -2.0f, 1.0f, 0.0f},
    {0.0f, 2.0f, 1.0f, -1.0f, 0.0f},
    {0.0f, -2.0f, 3.0f, -1.0f, 0.0f},
    {0.0f, -1.0f, 0.0f, 1.0f, 0.0f},
    {0.0f, 2.0f, -1.0f, -2.0f, 1.0f}};

constexpr double kG[5][3] = {
    {0.5, 0, 0},
    {0.5, 0.5, 0.5},
    {0.16666666666666666, -0.16666666666666666, 0.16666666666666666},
    {0.16666666666666666, 0.33333333333333331, 0.66666666666666663},
    {0, 0, 1}};

}  // namespace anx::wino33
