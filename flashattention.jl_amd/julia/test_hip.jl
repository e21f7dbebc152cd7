# test_hip.jl — the reference's own test relations (test/test.jl:5-21) run
# through the HIP binding, for a maintainer's machine with Julia + AMDGPU.jl
# and an MI355X (SURVEY §8f row 2).  Not executed in this repository (no Julia
# in the image); tests/test_gpu_*.py check the same relations through the
# Python ctypes mirror of the same C symbols.
#
#   julia --project -e 'using AMDGPU, FlashAttention; include("test_hip.jl")'
#
# with FlashAttentionHIP.jl included into FlashAttention (INTEGRATION.md).
using Test, NNlib, AMDGPU, FlashAttention

# test/test.jl:6-10 shape: Nq = Nkv = 30, dqk = 12, dv = 6, bs = 2
@testset "HIP dense_fa ≈ CPU dense_dpa ≈ NNlib (test/test.jl relations)" begin
    for T in (Float32, Float16, AMDGPU.BFloat16)
        q, k, v = rand(Float32, 30, 12, 2), rand(Float32, 30, 12, 2), rand(Float32, 30, 6, 2)
        y0, _ = dot_product_attention(permutedims(q, (2, 1, 3)), permutedims(k, (2, 1, 3)),
                                      permutedims(v, (2, 1, 3)))
        y1, _ = dense_dpa(q, k, v)                                        # CPU reference
        yd, ld, md = dense_fa(ROCArray(T.(q)), ROCArray(T.(k)), ROCArray(T.(v)))   # HIP
        y2 = Float32.(Array(yd))
        tol = T == Float32 ? sqrt(eps(Float32)) : 2f-2
        @test y1 ≈ permutedims(y0, (2, 1, 3))
        @test isapprox(y2, y1; rtol=tol)
        # l, m as the reference defines them (src/dense.jl:78-91)
        S = batched_mul(q, batched_transpose(k)) ./ sqrt(Float32(12))
        m = maximum(S; dims=2)
        l = sum(exp.(S .- m); dims=2)
        @test isapprox(Array(md), m; rtol=T == Float32 ? 1f-5 : 1f-3)
        @test isapprox(Array(ld), l; rtol=T == Float32 ? 1f-5 : 1f-3)
    end
end

# test/test.jl exactly as the reference runs it: Float64 arrays, Float64 `≈`
@testset "HIP dense_fa ≈ CPU dense_dpa in Float64 (test/test.jl:5-21)" begin
    q, k, v = rand(30, 12, 2), rand(30, 12, 2), rand(30, 6, 2)
    y1, _ = dense_dpa(q, k, v)
    yd, _, _ = dense_fa(ROCArray(q), ROCArray(k), ROCArray(v))
    @test Array(yd) ≈ y1
    Q, K, V, dO = (ROCArray(rand(64, 32, 2)) for _ in 1:4)
    O, l, m = dense_fa(Q, K, V)
    dQ, dK, dV = dense_fa_backward(Q, K, V, O, dO, l, m)
    @test eltype(dQ) == Float64
    @test isapprox(vec(sum(Array(dK); dims=1)), zeros(64); atol=1e-10)   # Σ_keys dK = 0
end

@testset "HIP windowed_fa / block_fa vs CPU windowed_dpa" begin
    x = rand(Float32, 16, 16, 8, 2)
    yc, _ = windowed_dpa(x, x, x, 4; stride=4, pad=0)
    yg, _, _ = windowed_fa(ROCArray(x), ROCArray(x), ROCArray(x), 4; stride=4, pad=0)
    @test isapprox(Array(yg), yc; rtol=sqrt(eps(Float32)))
    yb, _, _ = block_fa(ROCArray(x), ROCArray(x), ROCArray(x), 4)
    @test Array(yb) == Array(yg)
end

@testset "HIP dense_fa_backward: gradients sum to the reference identities" begin
    Q, K, V, dO = (ROCArray(rand(Float32, 64, 32, 2)) for _ in 1:4)
    O, l, m = dense_fa(Q, K, V)
    dQ, dK, dV = FlashAttention.dense_fa_backward(Q, K, V, O, dO, l, m)
    @test isapprox(vec(sum(Array(dV); dims=1)), vec(sum(Array(dO); dims=1)); rtol=1f-4)   # rows of P sum to 1
    @test maximum(abs, sum(Array(dK); dims=1)) < 1f-3 * maximum(abs, Array(dK)) * 64      # Σ_keys dS = 0
end

@testset "HIP fused_softmax! ≈ NNlib.softmax" begin
    S = rand(Float32, 37, 5, 2)
    @test isapprox(Array(fused_softmax(ROCArray(S); dims=1)), NNlib.softmax(S; dims=1); rtol=1f-5)
    @test isapprox(Array(fused_softmax(ROCArray(S); dims=2)), NNlib.softmax(S; dims=2); rtol=1f-5)
end
