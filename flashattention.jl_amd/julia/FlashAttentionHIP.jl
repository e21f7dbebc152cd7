# FlashAttentionHIP.jl — ccall binding of libfa_hip.so (MI355X / gfx950) for
# nikopj/FlashAttention.jl.
#
# Include from src/FlashAttention.jl next to the disabled CUDA include
# (reference src/FlashAttention.jl:29):
#
#     using AMDGPU
#     include("hip/FlashAttentionHIP.jl")
#
# It adds methods for AMDGPU device arrays (ROCArray) to the reference's own
# generic functions, exactly like the CUDA precedent
# `dense_fa!(O::CuArray{T,3}, …)` (src/cuda/flash.jl:121-140), so user code
# calling dense_fa / dense_fa! / windowed_fa / block_fa on ROCArrays runs on
# the HIP kernels with no other change.  Arrays keep Julia's column-major
# layout; the C ABI (include/fa_hip.h) consumes it as is — no copies.
#
# NOT EXECUTED in this repository's CI (no Julia in the image); the Python
# ctypes mirror (flashattention.jl_amd/fa_hip) binds the same symbols and
# carries the parity tests.

const libfa_hip = get(ENV, "FA_HIP_LIB", joinpath(@__DIR__, "..", "libfa_hip.so"))

const FA_DTYPE = Dict(Float32 => Cint(0), AMDGPU.BFloat16 => Cint(1), Float16 => Cint(2), Float64 => Cint(3))

fa_dtype(::Type{T}) where {T} = haskey(FA_DTYPE, T) ? FA_DTYPE[T] :
    throw(ArgumentError("FlashAttentionHIP: element type $T not supported (Float64, Float32, Float16, BFloat16)"))

function fa_check(rc::Cint)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:fa_last_error, libfa_hip), Cstring, ()))
    rc == 1 && occursin("DimensionMismatch", msg) && throw(DimensionMismatch(msg))
    error("libfa_hip: ", msg)
end

stream_ptr() = AMDGPU.stream().stream   # hipStream_t of the task-local stream

# Scratch for the C ABI's workspace arguments: ONE buffer per device, grown on demand and
# shared by every call on that device, whatever task or stream makes it (task-local
# streams come and go with their tasks; a cache keyed by stream would keep one buffer per
# stream ever seen, each up to the largest workspace a call needed on it).  Use is
# stream-ordered: every call records an event on its stream after its launches, and a
# call on another stream first makes its own stream wait on that event (no host
# synchronisation), so two streams never hold the buffer at once.  Growing synchronises
# the current stream (which already waits on the previous user) before the old buffer is
# freed.  Memory: the largest workspace any call on the device needed — e.g. 0.54 GB for
# configs[3]'s backward (two chains of running dQ sums), 17.2 GB for configs[4]'s
# 1024 slabs on one GPU.  free_workspaces!() gives it all back.
const libhip = "libamdhip64"
hip_check(rc::Cint) = rc == 0 ? nothing : error("HIP runtime error $rc")

mutable struct Scratch
    buf::ROCArray{UInt8,1}
    last::UInt                # hipStream_t of the last call that used buf
    ev::Ptr{Cvoid}            # hipEvent_t recorded on that stream after its launches
end
const _WS = Dict{Int,Scratch}()
const _WS_LOCK = ReentrantLock()

# f(ws) with this device's scratch buffer of at least nbytes; f enqueues on stream_ptr()
function with_workspace(f, nbytes::Integer)
    n = max(Int(nbytes), 1)
    dev = AMDGPU.device_id(AMDGPU.device())
    s = stream_ptr()
    lock(_WS_LOCK) do
        e = get(_WS, dev, nothing)
        if e === nothing
            ev = Ref{Ptr{Cvoid}}(C_NULL)
            hip_check(ccall((:hipEventCreateWithFlags, libhip), Cint, (Ref{Ptr{Cvoid}}, Cuint), ev, 0x2))  # DisableTiming
            e = Scratch(ROCArray{UInt8}(undef, n), UInt(s), ev[])
            _WS[dev] = e
        elseif e.last != UInt(s)
            # the event was recorded on the previous user's stream after its launches
            hip_check(ccall((:hipStreamWaitEvent, libhip), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cuint), s, e.ev, 0))
            e.last = UInt(s)
        end
        if length(e.buf) < n
            hip_check(ccall((:hipStreamSynchronize, libhip), Cint, (Ptr{Cvoid},), s))
            AMDGPU.unsafe_free!(e.buf)
            e.buf = ROCArray{UInt8}(undef, n)
        end
        r = f(e.buf)
        hip_check(ccall((:hipEventRecord, libhip), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), e.ev, s))
        r
    end
end

# Frees every cached scratch buffer (after the work that used them has finished).
function free_workspaces!()
    lock(_WS_LOCK) do
        for (_, e) in _WS
            hip_check(ccall((:hipEventSynchronize, libhip), Cint, (Ptr{Cvoid},), e.ev))
            AMDGPU.unsafe_free!(e.buf)
            hip_check(ccall((:hipEventDestroy, libhip), Cint, (Ptr{Cvoid},), e.ev))
        end
        empty!(_WS)
    end
    nothing
end

# dense_fa!(O, l, m, Q, K, V) — replaces the body of src/dense.jl:21-102, with the
# kernels' own statistics type (Float32 l, m)
function dense_fa_f32!(O::ROCArray{T,3}, l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                       Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}) where {T}
    N, d, B = size(Q)
    Nk, dv = size(K, 1), size(V, 2)
    size(K) == (Nk, d, B) || throw(DimensionMismatch("K"))
    size(V) == (Nk, dv, B) || throw(DimensionMismatch("V"))
    size(O) == (N, dv, B) || throw(DimensionMismatch("O"))
    size(l) == (N, 1, B) && size(m) == (N, 1, B) || throw(DimensionMismatch("l, m must be (N, 1, batch)"))
    nws = ccall((:fa_dense_fwd_workspace, libfa_hip), Csize_t,
                (Cint, Int64, Int64, Int64, Int64, Int64), fa_dtype(T), N, Nk, d, dv, B)
    if nws == 0
        fa_check(ccall((:fa_dense_fwd, libfa_hip), Cint,
                       (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32},
                        Int64, Int64, Int64, Int64, Int64, Cfloat, Ptr{Cvoid}),
                       fa_dtype(T), Q, K, V, O, l, m, N, Nk, d, dv, B, 0f0, stream_ptr()))
    else   # ragged Nk: zero-padded K / V copies in the workspace let the fast kernels run
        with_workspace(nws) do ws
            fa_check(ccall((:fa_dense_fwd_ws, libfa_hip), Cint,
                           (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32},
                            Int64, Int64, Int64, Int64, Int64, Cfloat, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                           fa_dtype(T), Q, K, V, O, l, m, N, Nk, d, dv, B, 0f0, ws, nws, stream_ptr()))
        end
    end
    return O, l, m
end

# l, m in another element type — what the reference's own wrapper allocates,
# `l = similar(Q, N, 1, B)` (src/dense.jl:12-13), i.e. T itself for Float64, Float16 and
# BFloat16 inputs.  The C ABI writes float32 statistics: they are staged in Float32 and
# converted on the device (for Float64 the kernels keep l, m in double internally and
# round them to Float32 at this boundary, DESIGN.md §3).
function dense_fa_staged!(O::ROCArray{T,3}, l::ROCArray{S,3}, m::ROCArray{S,3},
                          Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}) where {T,S}
    size(l) == size(m) || throw(DimensionMismatch("l, m"))
    lf, mf = similar(l, Float32), similar(m, Float32)
    dense_fa_f32!(O, lf, mf, Q, K, V)
    l .= lf
    m .= mf
    return O, l, m
end

# Methods on the reference's generic function.  Dispatch by construction: for every call
# the methods that apply include one that is a subtype of all the others, the
# reference's `dense_fa!(O::AbstractArray{T,3}, l::AbstractArray{T,3}, …) where {T}`
# (src/dense.jl:21-27) included, so no call is ambiguous
# (tests/test_julia_binding.py::test_dispatch_has_a_most_specific_hip_method).
#   T data, Float32 statistics (the C ABI's types)
function dense_fa!(O::ROCArray{T,3}, l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                   Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}) where {T}
    return dense_fa_f32!(O, l, m, Q, K, V)
end
#   everything of one type T: a strict subtype of the reference's method
function dense_fa!(O::ROCArray{T,3}, l::ROCArray{T,3}, m::ROCArray{T,3},
                   Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}) where {T}
    return dense_fa_staged!(O, l, m, Q, K, V)
end
#   everything Float32: the three methods above and the reference's all apply
function dense_fa!(O::ROCArray{Float32,3}, l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                   Q::ROCArray{Float32,3}, K::ROCArray{Float32,3}, V::ROCArray{Float32,3})
    return dense_fa_f32!(O, l, m, Q, K, V)
end
#   any other statistics type S
function dense_fa!(O::ROCArray{T,3}, l::ROCArray{S,3}, m::ROCArray{S,3},
                   Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}) where {T,S}
    return dense_fa_staged!(O, l, m, Q, K, V)
end

# dense_fa(q, k, v) — src/dense.jl:1-19 (l, m are Float32 on the device: DESIGN.md)
function dense_fa(q::ROCArray{T,D}, k::ROCArray{T,D}, v::ROCArray{T,D}) where {T,D}
    d, dv, B = size(q, D - 1), size(v, D - 1), size(q, D)
    Q, K, V = reshape(q, :, d, B), reshape(k, :, d, B), reshape(v, :, dv, B)
    N = size(Q, 1)
    O = similar(Q, N, dv, B)                      # dv, not d (reference bug A.1 not inherited)
    l = similar(Q, Float32, N, 1, B)
    m = similar(Q, Float32, N, 1, B)
    dense_fa!(O, l, m, Q, K, V)
    return reshape(O, size(q)[1:D-2]..., dv, :), l, m
end

# dense_fa_backward(Q, K, V, O, dO, l, m) — src/dense.jl:104-167
# `handoff`: optional Ref{Cint} that receives fa_dense_bwd_handoff_status after the call
# (-1 two-pass form, 0 single pass completed, 1 a slab's dQ hand-off gave up and its dQ was
# recomputed); it synchronises the stream.
function dense_fa_backward_f32(Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3},
                               O::ROCArray{T,3}, dO::ROCArray{T,3},
                               l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                               handoff::Union{Nothing,Base.RefValue{Cint}}) where {T}
    N, d, B = size(Q)
    Nk, dv = size(K, 1), size(V, 2)
    size(K) == (Nk, d, B) && size(V) == (Nk, dv, B) ||
        throw(DimensionMismatch("K, V shapes disagree with Q"))
    size(O) == (N, dv, B) && size(dO) == (N, dv, B) ||
        throw(DimensionMismatch("O, dO must be (N, dv, batch)"))
    size(l) == (N, 1, B) && size(m) == (N, 1, B) ||
        throw(DimensionMismatch("l, m must be (N, 1, batch)"))
    dQ, dK, dV = similar(Q), similar(K), similar(V)
    nws = ccall((:fa_dense_bwd_workspace, libfa_hip), Csize_t,
                (Cint, Int64, Int64, Int64, Int64, Int64), fa_dtype(T), N, Nk, d, dv, B)
    with_workspace(nws) do ws
        fa_check(ccall((:fa_dense_bwd, libfa_hip), Cint,
                       (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32},
                        Ptr{Float32}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid},
                        Int64, Int64, Int64, Int64, Int64, Cfloat, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                       fa_dtype(T), Q, K, V, O, dO, l, m, dQ, dK, dV, N, Nk, d, dv, B, 0f0,
                       ws, nws, stream_ptr()))
        if handoff !== nothing
            fa_check(ccall((:fa_dense_bwd_handoff_status, libfa_hip), Cint,
                           (Ptr{Cvoid}, Csize_t, Ptr{Cvoid}, Ptr{Cint}), ws, nws, stream_ptr(), handoff))
        end
    end
    return dQ, dK, dV
end

# Methods on the reference's generic function (src/dense.jl:104-111, `… l, m ::
# AbstractArray{T,3}) where T`), laid out as dense_fa!'s: T data with Float32 statistics,
# one type T throughout, all Float32, any other statistics type S.
function dense_fa_backward(Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3},
                           O::ROCArray{T,3}, dO::ROCArray{T,3},
                           l::ROCArray{Float32,3}, m::ROCArray{Float32,3};
                           handoff::Union{Nothing,Base.RefValue{Cint}}=nothing) where {T}
    return dense_fa_backward_f32(Q, K, V, O, dO, l, m, handoff)
end
function dense_fa_backward(Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3},
                           O::ROCArray{T,3}, dO::ROCArray{T,3},
                           l::ROCArray{T,3}, m::ROCArray{T,3};
                           handoff::Union{Nothing,Base.RefValue{Cint}}=nothing) where {T}
    return dense_fa_backward_f32(Q, K, V, O, dO, Float32.(l), Float32.(m), handoff)
end
function dense_fa_backward(Q::ROCArray{Float32,3}, K::ROCArray{Float32,3}, V::ROCArray{Float32,3},
                           O::ROCArray{Float32,3}, dO::ROCArray{Float32,3},
                           l::ROCArray{Float32,3}, m::ROCArray{Float32,3};
                           handoff::Union{Nothing,Base.RefValue{Cint}}=nothing)
    return dense_fa_backward_f32(Q, K, V, O, dO, l, m, handoff)
end
function dense_fa_backward(Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3},
                           O::ROCArray{T,3}, dO::ROCArray{T,3},
                           l::ROCArray{S,3}, m::ROCArray{S,3};
                           handoff::Union{Nothing,Base.RefValue{Cint}}=nothing) where {T,S}
    return dense_fa_backward_f32(Q, K, V, O, dO, Float32.(l), Float32.(m), handoff)
end

# windowed_fa(q, k, v, ws; stride, pad) — src/windowed.jl:3-23 (fused on the device)
function windowed_fa(q::ROCArray{T,N}, k::ROCArray{T,N}, v::ROCArray{T,N}, windowsize;
                     stride=windowsize, pad=(windowsize - 1) ÷ 2) where {T,N}
    nsp = N - 2
    spatial = Int64[size(q, i) for i in 1:nsp]
    d, dv, B = size(q, N - 1), size(v, N - 1), size(q, N)
    L = prod((s + 2pad - windowsize) ÷ stride + 1 for s in spatial)
    y = similar(v, size(q)[1:N-2]..., dv, B)
    l = similar(q, Float32, windowsize^nsp, 1, L, B)
    m = similar(q, Float32, windowsize^nsp, 1, L, B)
    nws = ccall((:fa_windowed_fwd_workspace, libfa_hip), Csize_t,
                (Cint, Cint, Ptr{Int64}, Int64, Int64, Int64, Int64, Int64, Int64),
                fa_dtype(T), nsp, spatial, d, dv, B, windowsize, stride, pad)
    with_workspace(nws) do ws
        fa_check(ccall((:fa_windowed_fwd, libfa_hip), Cint,
                       (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32},
                        Cint, Ptr{Int64}, Int64, Int64, Int64, Int64, Int64, Int64, Cfloat,
                        Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                       fa_dtype(T), q, k, v, y, l, m, nsp, spatial, d, dv, B, windowsize, stride, pad,
                       0f0, ws, nws, stream_ptr()))
    end
    return y, l, m
end

# windowed_fa_backward(q, k, v, y, dy, l, m, ws; stride, pad) — the chain rule of
# windowed_fa (SURVEY §8f row 1; the reference README claims it, no code exists)
function windowed_fa_backward(q::ROCArray{T,N}, k::ROCArray{T,N}, v::ROCArray{T,N},
                              y::ROCArray{T,N}, dy::ROCArray{T,N},
                              l::ROCArray{Float32}, m::ROCArray{Float32}, windowsize;
                              stride=windowsize, pad=(windowsize - 1) ÷ 2) where {T,N}
    nsp = N - 2
    spatial = Int64[size(q, i) for i in 1:nsp]
    d, dv, B = size(q, N - 1), size(v, N - 1), size(q, N)
    L = prod((s + 2pad - windowsize) ÷ stride + 1 for s in spatial)
    size(k) == size(q) || throw(DimensionMismatch("k must have q's shape"))
    size(v)[1:nsp] == size(q)[1:nsp] && size(v, N) == B ||
        throw(DimensionMismatch("v must share q's spatial dims and batch"))
    size(y) == size(v) && size(dy) == size(v) ||
        throw(DimensionMismatch("y and dy must have v's shape (spatial..., dv, batch)"))
    size(l) == (windowsize^nsp, 1, L, B) && size(m) == (windowsize^nsp, 1, L, B) ||
        throw(DimensionMismatch("l, m must be (ws^k, 1, L, batch), the forward's window statistics"))
    dq, dk, dv_ = similar(q), similar(k), similar(v)
    nws = ccall((:fa_windowed_workspace, libfa_hip), Csize_t,
                (Cint, Cint, Ptr{Int64}, Int64, Int64, Int64, Int64, Int64, Int64),
                fa_dtype(T), nsp, spatial, d, dv, B, windowsize, stride, pad)
    with_workspace(nws) do ws
        fa_check(ccall((:fa_windowed_bwd, libfa_hip), Cint,
                       (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32},
                        Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Int64}, Int64, Int64, Int64, Int64, Int64, Int64,
                        Cfloat, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                       fa_dtype(T), q, k, v, y, dy, l, m, dq, dk, dv_, nsp, spatial, d, dv, B,
                       windowsize, stride, pad, 0f0, ws, nws, stream_ptr()))
    end
    return dq, dk, dv_
end

# window(x, ws; stride, pad) / unwindow(X, size(x), ws; stride, pad) — src/utils.jl:36-54
# (NNlib.unfold / NNlib.fold, the sum over overlapping windows) on the device
function window(x::ROCArray{T,N}, windowsize; stride=windowsize, pad=(windowsize - 1) ÷ 2) where {T,N}
    nsp = N - 2
    spatial = Int64[size(x, i) for i in 1:nsp]
    C, B = size(x, N - 1), size(x, N)
    L = prod((s + 2pad - windowsize) ÷ stride + 1 for s in spatial)
    X = similar(x, windowsize^nsp, C, L, B)
    fa_check(ccall((:fa_window, libfa_hip), Cint,
                   (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Int64}, Int64, Int64, Int64, Int64, Int64, Ptr{Cvoid}),
                   fa_dtype(T), x, X, nsp, spatial, C, B, windowsize, stride, pad, stream_ptr()))
    return X
end
function unwindow(X::ROCArray{T,4}, outputsize::NTuple{N}, windowsize;
                  stride=windowsize, pad=(windowsize - 1) ÷ 2) where {T,N}
    nsp = N - 2
    spatial = Int64[outputsize[i] for i in 1:nsp]
    C, B = size(X, 2), size(X, 4)
    x = similar(X, outputsize...)
    fa_check(ccall((:fa_unwindow, libfa_hip), Cint,
                   (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Int64}, Int64, Int64, Int64, Int64, Int64, Ptr{Cvoid}),
                   fa_dtype(T), X, x, nsp, spatial, C, B, windowsize, stride, pad, stream_ptr()))
    return x
end

fa_abi_version() = ccall((:fa_abi_version, libfa_hip), Cint, ())
fa_max_head_dim() = ccall((:fa_max_head_dim, libfa_hip), Cint, ())

# block_fa — src/windowed.jl:1
block_fa(q::ROCArray, k::ROCArray, v::ROCArray, windowsize; pad=0) =
    windowed_fa(q, k, v, windowsize; stride=windowsize, pad=pad)

# circulant_fa!(O, l, m, Q, K, V, W) — replaces src/circulant.jl:9-118
function circulant_fa_f32!(O::ROCArray{T,3}, l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                           Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}, W::Int) where {T}
    N, d, B = size(Q)
    dv = size(V, 2)
    size(K) == (N, d, B) || throw(DimensionMismatch("K"))
    size(V) == (N, dv, B) || throw(DimensionMismatch("V"))
    size(O) == (N, dv, B) || throw(DimensionMismatch("O"))
    size(l) == (N, 1, B) && size(m) == (N, 1, B) || throw(DimensionMismatch("l, m must be (N, 1, batch)"))
    fa_check(ccall((:fa_circulant_fwd, libfa_hip), Cint,
                   (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32},
                    Int64, Int64, Int64, Int64, Int64, Cfloat, Ptr{Cvoid}),
                   fa_dtype(T), Q, K, V, O, l, m, N, d, dv, B, W, 0f0, stream_ptr()))
    return O, l, m
end

# l, m in another element type, staged in Float32 as dense_fa_staged! does
function circulant_fa_staged!(O::ROCArray{T,3}, l::ROCArray{S,3}, m::ROCArray{S,3},
                              Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}, W::Int) where {T,S}
    size(l) == size(m) || throw(DimensionMismatch("l, m"))
    lf, mf = similar(l, Float32), similar(m, Float32)
    circulant_fa_f32!(O, lf, mf, Q, K, V, W)
    l .= lf
    m .= mf
    return O, l, m
end

# Methods on the reference's generic function (src/circulant.jl:9-16, `… ::AbstractArray{T,3},
# W::Int) where {T}`), laid out as dense_fa!'s.
function circulant_fa!(O::ROCArray{T,3}, l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                       Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}, W::Int) where {T}
    return circulant_fa_f32!(O, l, m, Q, K, V, W)
end
function circulant_fa!(O::ROCArray{T,3}, l::ROCArray{T,3}, m::ROCArray{T,3},
                       Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}, W::Int) where {T}
    return circulant_fa_staged!(O, l, m, Q, K, V, W)
end
function circulant_fa!(O::ROCArray{Float32,3}, l::ROCArray{Float32,3}, m::ROCArray{Float32,3},
                       Q::ROCArray{Float32,3}, K::ROCArray{Float32,3}, V::ROCArray{Float32,3}, W::Int)
    return circulant_fa_f32!(O, l, m, Q, K, V, W)
end
function circulant_fa!(O::ROCArray{T,3}, l::ROCArray{S,3}, m::ROCArray{S,3},
                       Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}, W::Int) where {T,S}
    return circulant_fa_staged!(O, l, m, Q, K, V, W)
end

# circulant_fa(Q, K, V, W) — src/circulant.jl:1-7, passing W (the reference call drops it)
function circulant_fa(Q::ROCArray{T,3}, K::ROCArray{T,3}, V::ROCArray{T,3}, W::Int) where {T}
    N, _, B = size(Q)
    O = similar(V, N, size(V, 2), B)
    l = similar(Q, Float32, N, 1, B)
    m = similar(Q, Float32, N, 1, B)
    return circulant_fa!(O, l, m, Q, K, V, W)
end

# fused_softmax!(P, S; dims) — replaces src/fused_softmax.jl:10-15 (and the CUDA
# versions src/cuda/fused_softmax.jl) for device arrays; P may be S
function fused_softmax!(P::ROCArray{T,3}, S::ROCArray{T,3}; dims=1) where {T}
    dims in (1, 2) || throw(ArgumentError("only softmax in dims 1 or 2 supported"))
    size(P) == size(S) || throw(DimensionMismatch("P and S must have the same size"))
    M, N, B = size(S)
    nws = ccall((:fa_softmax_workspace, libfa_hip), Csize_t, (Int64, Int64, Int64, Cint), M, N, B, dims)
    with_workspace(nws) do ws
        fa_check(ccall((:fa_softmax, libfa_hip), Cint,
                       (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Int64, Int64, Cint, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                       fa_dtype(T), S, P, M, N, B, dims, ws, nws, stream_ptr()))
    end
    return P
end
fused_softmax!(P::ROCArray{T,2}, S::ROCArray{T,2}; dims=1) where {T} =
    (fused_softmax!(reshape(P, size(P)..., 1), reshape(S, size(S)..., 1); dims=dims); P)
fused_softmax(S::ROCArray; dims=1) = fused_softmax!(similar(S), S; dims=dims)
