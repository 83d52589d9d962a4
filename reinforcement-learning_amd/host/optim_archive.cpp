// optim_archive.cpp -- <NAME>_OPTIM.lt, the reference's optimizer checkpoint (GGL::Model::Save / Load,
// GigaLearnCPP/src/private/GigaLearnCPP/Util/Models.cpp:116-126,168-186): written and read by libtorch's
// own torch::optim::AdamW::save / load through a torch::serialize archive, exactly as the reference
// does, so the file is byte-for-byte the format its Model::Load expects (state keyed by parameter
// address, mapped back by parameter order on load).  Built against the libtorch of the installed
// PyTorch (plumbing); rlgpu/checkpoint.py drives it.
//
// It also writes and reads the model archives <NAME>.lt (GGL::Model::Save / Load, Models.cpp:116-166): the
// Sequential GGL::Model builds (Models.cpp:7-33: per hidden layer Linear, LayerNorm, LeakyReLU; then the output
// Linear unless out is 0, the shared head's addOutputLayer = false) saved with torch::save(seq, stream) and
// read with torch::load(seq, stream), with Model::Load's parameter-size check.
//
// usage: rlgpu_optim_lt save <out.lt> <state.f32> <step> <lr> <beta1> <beta2> <eps> <weight_decay> <shape>...
//        rlgpu_optim_lt load <in.lt> <state.f32> <shape>...
//        rlgpu_optim_lt model-save <out.lt> <params.f32> <obs> <out> <h1> [h2 ...]
//        rlgpu_optim_lt model-load <in.lt> <params.f32> <obs> <out> <h1> [h2 ...]
//   params.f32: the model's parameters flat in parameters() order (model-load writes them).
//   shape: dimensions joined by 'x' (e.g. 384x167), one per model parameter in parameters() order;
//   state.f32: every parameter's exp_avg (flat, parameter order), then every exp_avg_sq.  load writes
//   it preceded by the step as an int64 (0 and zero moments for parameters without state).
#include <torch/torch.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

namespace {

std::vector<int64_t> parse_shape(const std::string& s) {
    std::vector<int64_t> d;
    size_t p = 0;
    while (p <= s.size()) {
        size_t q = s.find('x', p);
        if (q == std::string::npos) q = s.size();
        d.push_back(std::stoll(s.substr(p, q - p)));
        p = q + 1;
    }
    return d;
}

std::vector<torch::Tensor> make_params(char** shapes, int n) {
    std::vector<torch::Tensor> ps;
    for (int i = 0; i < n; i++) ps.push_back(torch::zeros(parse_shape(shapes[i])));
    return ps;
}

torch::nn::Sequential make_model(int obs, int out, const std::vector<int>& layers) {
    torch::nn::Sequential seq;
    int last = obs;
    for (int h : layers) {
        seq->push_back(torch::nn::Linear(last, h));
        seq->push_back(torch::nn::LayerNorm(torch::nn::LayerNormOptions({(int64_t)h})));
        last = h;
        seq->push_back(torch::nn::LeakyReLU());
    }
    if (out > 0) seq->push_back(torch::nn::Linear(last, out));
    return seq;
}

std::vector<int64_t> seq_sizes(torch::nn::Sequential& seq) {  // GetSeqSizes (Models.cpp:79-87)
    std::vector<int64_t> r;
    for (size_t i = 0; i < seq->size(); i++)
        for (auto& p : seq[i]->parameters()) r.push_back(p.numel());
    return r;
}

int model_mode(bool save, int argc, char** argv) {
    if (argc < 7) return 2;
    std::vector<int> layers;
    for (int i = 6; i < argc; i++) layers.push_back(std::atoi(argv[i]));
    torch::nn::Sequential seq = make_model(std::atoi(argv[4]), std::atoi(argv[5]), layers);
    torch::NoGradGuard ng;
    int64_t total = 0;
    for (auto& p : seq->parameters()) total += p.numel();
    std::vector<float> buf((size_t)total);
    if (save) {
        std::ifstream in(argv[3], std::ios::binary);
        in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float)));
        if (!in) {
            std::cerr << "parameter file too short\n";
            return 3;
        }
        int64_t off = 0;
        for (auto& p : seq->parameters()) {
            p.copy_(torch::from_blob(buf.data() + off, p.sizes(), torch::kFloat32));
            off += p.numel();
        }
        std::ofstream out(argv[2], std::ios::binary);  // Model::Save (Models.cpp:116-120)
        torch::save(seq, out);
        return out ? 0 : 3;
    }
    const auto before = seq_sizes(seq);
    std::ifstream in(argv[2], std::ios::binary);  // Model::Load (Models.cpp:130-166)
    in >> std::noskipws;
    if (!in.good()) {
        std::cerr << "cannot open " << argv[2] << "\n";
        return 3;
    }
    torch::load(seq, in);
    if (seq_sizes(seq) != before) {
        std::cerr << "Saved model has different size than current model, cannot load model from " << argv[2] << "\n";
        return 5;
    }
    int64_t off = 0;
    for (auto& p : seq->parameters()) {
        auto c = p.to(torch::kCPU).to(torch::kFloat32).contiguous();
        std::copy(c.data_ptr<float>(), c.data_ptr<float>() + c.numel(), buf.begin() + off);
        off += p.numel();
    }
    std::ofstream out(argv[3], std::ios::binary);
    out.write(reinterpret_cast<const char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float)));
    return out ? 0 : 3;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        if (argc < 4) return 2;
        const std::string mode = argv[1];
        if (mode == "model-save" || mode == "model-load") return model_mode(mode == "model-save", argc, argv);
        if (mode == "save") {
            if (argc < 10) return 2;
            const int64_t step = std::atoll(argv[4]);
            const double lr = std::atof(argv[5]), b1 = std::atof(argv[6]), b2 = std::atof(argv[7]), eps = std::atof(argv[8]),
                         wd = std::atof(argv[9]);
            std::vector<torch::Tensor> ps = make_params(argv + 10, argc - 10);
            int64_t total = 0;
            for (auto& p : ps) total += p.numel();
            std::vector<float> buf((size_t)(2 * total));
            std::ifstream in(argv[3], std::ios::binary);
            in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float)));
            if (!in) {
                std::cerr << "state file too short\n";
                return 3;
            }
            // Model::Model: MakeOptimizer(AdamW, parameters(), lr) (Models.h:40-56)
            torch::optim::AdamW opt(ps, torch::optim::AdamWOptions(lr).betas({b1, b2}).eps(eps).weight_decay(wd));
            int64_t off = 0;
            for (auto& p : ps) {
                auto st = std::make_unique<torch::optim::AdamWParamState>();
                st->step(step);
                st->exp_avg(torch::from_blob(buf.data() + off, p.sizes(), torch::kFloat32).clone());
                st->exp_avg_sq(torch::from_blob(buf.data() + total + off, p.sizes(), torch::kFloat32).clone());
                opt.state()[p.unsafeGetTensorImpl()] = std::move(st);
                off += p.numel();
            }
            torch::serialize::OutputArchive archive;  // Model::Save (Models.cpp:122-125)
            opt.save(archive);
            archive.save_to(argv[2]);
            return 0;
        }
        if (mode == "load") {
            std::vector<torch::Tensor> ps = make_params(argv + 4, argc - 4);
            torch::optim::AdamW opt(ps, torch::optim::AdamWOptions(1e-3));
            torch::serialize::InputArchive archive;  // Model::Load (Models.cpp:177-180)
            archive.load_from(argv[2]);
            opt.load(archive);
            int64_t step = 0, total = 0;
            for (auto& p : ps) total += p.numel();
            std::vector<float> buf((size_t)(2 * total), 0.f);
            int64_t off = 0;
            for (auto& p : ps) {
                auto it = opt.state().find(p.unsafeGetTensorImpl());
                if (it != opt.state().end()) {
                    auto& st = static_cast<torch::optim::AdamWParamState&>(*it->second);
                    step = st.step();
                    auto m = st.exp_avg().to(torch::kCPU).to(torch::kFloat32).contiguous();
                    auto v = st.exp_avg_sq().to(torch::kCPU).to(torch::kFloat32).contiguous();
                    if (m.numel() != p.numel() || v.numel() != p.numel()) {
                        std::cerr << "optimizer state does not match the parameter shapes\n";
                        return 3;
                    }
                    std::copy(m.data_ptr<float>(), m.data_ptr<float>() + m.numel(), buf.begin() + off);
                    std::copy(v.data_ptr<float>(), v.data_ptr<float>() + v.numel(), buf.begin() + total + off);
                }
                off += p.numel();
            }
            std::ofstream out(argv[3], std::ios::binary);
            out.write(reinterpret_cast<const char*>(&step), sizeof step);
            out.write(reinterpret_cast<const char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float)));
            return out ? 0 : 3;
        }
        return 2;
    } catch (const std::exception& e) {
        std::cerr << e.what() << "\n";
        return 4;
    }
}
