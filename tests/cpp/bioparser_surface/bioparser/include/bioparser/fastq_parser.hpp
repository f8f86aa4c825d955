// TEST-ONLY: see parser.hpp.
#pragma once
#include "parser.hpp"
namespace bioparser {
template <class T>
class FastqParser : public SurfaceParser<T> {
public:
    using SurfaceParser<T>::SurfaceParser;
};
}  // namespace bioparser
